"""CPU tests of the round harness (flpytorch_amd/harness.py) — its orchestration, not the kernels.

The harness is driven with test doubles of the codec and fold protocols backed by the ORACLE
(oracle/codecs.py: the reference's compressVector / serverGradient restated op for op), so the
sampling order, the per-client pattern + seed draws on the shared stream, the local SGD step and the
history scalars are checked here against the reference's own runs (tests/golden/harness.json, from
make_golden_harness.py).  The product path (HIP codecs + HIP fold) is tests/test_gpu_harness.py.
"""
import numpy as np
import pytest
import torch

from oracle import codecs as oc
from tests.harness_cases import DATA, META, RUN_NAMES, check_history, check_server_shift, simulation


class OracleCompressorDouble:
    """The reference's Compressor protocol over the oracle (CPU tensors in and out)."""

    def __init__(self, spec, D):
        self.o = oc.OracleCompressor(spec, D)
        self.last_need_to_send_advance = 0

    def isUnbiasedCompressor(self):
        return hasattr(self.o, "w")

    def isContractionCompressor(self):
        return hasattr(self.o, "alpha")

    def getW(self):
        return self.o.w

    def getAlphaContraction(self):
        return self.o.alpha

    def generateCompressPattern(self, rndgen, device, clientId, H):
        self.o.generate(rndgen)

    def compressVector(self, x):
        out = self.o.compress(x.detach().cpu().numpy())
        self.last_need_to_send_advance = self.o.last_need_to_send_advance
        return torch.from_numpy(np.ascontiguousarray(out))


def oracle_server_gradient(buf, clients, model, x, H):
    rows, w = [], []
    for i in range(clients):
        buf.waitForItem()
        r = buf.get(i)
        rows.append(r["model"].cpu().numpy())
        w.append(r["client_state"]["weight"])
    return torch.from_numpy(oc.server_gradient(x.cpu().numpy(), rows, w))


def oracle_server_gradient_diana(buf, clients, model, x, H):
    gs = oracle_server_gradient(buf, clients, model, x, H)
    H["m"] = gs
    return H["h"] + gs                                                   # algorithms.py:1419-1421


def oracle_diana_step(comp, g, h, alpha):
    m = comp.compressVector(g - h)                                       # algorithms.py:1386-1391
    return m, h + alpha * m


def oracle_ef21_step(comp, g, g_prev):
    mult = 1.0 if comp.isContractionCompressor() else 1.0 / (1.0 + comp.getW())
    return g_prev + comp.compressVector(g - g_prev) * mult               # algorithms.py:1508-1513


def oracle_marina_step(comp, g, g_old, g_prev):
    return g_prev + comp.compressVector(g - g_old)                       # algorithms.py:536-537


def oracle_simulation(name, **kw):
    fold = oracle_server_gradient_diana if META[name]["algorithm"] == "diana" else oracle_server_gradient
    return simulation(name, "cpu", init_compressor=OracleCompressorDouble, server_gradient=fold,
                      diana_step=oracle_diana_step, ef21_step=oracle_ef21_step, marina_step=oracle_marina_step,
                      **kw)


def run_collecting_shift(sim):
    """sim.run(), keeping DIANA's server shift after every round."""
    hs = []
    for r in range(sim.rounds):
        sim.run_round(r)
        if "h" in sim.H:
            hs.append(sim.H["h"].detach().cpu().numpy().copy())
    return sim.H, hs


@pytest.mark.parametrize("name", RUN_NAMES)
def test_harness_replays_reference_runs(name):
    sim = oracle_simulation(name, record_iterates=True)
    H, hs = run_collecting_shift(sim)
    check_history(name, H)
    if META[name]["algorithm"] == "diana":
        check_server_shift(name, hs)
    # the iterate after every round's global step
    for r in range(META[name]["rounds"]):
        np.testing.assert_allclose(sim.iterates[r].numpy(), DATA[f"{name}_iterates"][r], rtol=1e-6, atol=1e-7,
                                   err_msg=f"{name} round {r}")


def test_sampling_matches_numpy_stream():
    from flpytorch_amd import harness
    rs, ref = np.random.RandomState(456), np.random.RandomState(456)
    got = harness.get_sampled_clients(10, 3, 5, rs)
    want = [ref.choice(10, 3, replace=False) for _ in range(5)]
    assert all(np.array_equal(a, b) for a, b in zip(got, want))
    rs, ref = np.random.RandomState(9), np.random.RandomState(9)
    got = harness.get_sampled_clients(6, None, 4, rs, sampling="poisson", poisson_p=0.3)
    want = [np.asarray([j for j in range(6) if ref.uniform() < 0.3]) for _ in range(4)]
    assert all(np.array_equal(a, b) for a, b in zip(got, want))
    with pytest.raises(AssertionError):
        harness.get_sampled_clients(6, 2, 1, rs, sampling="stratified")


def test_dense_model_gradient_matches_autograd_module():
    """DenseModel on a flat vector == the reference's nn.Sequential "dense" model
    (model_funcs.py:170-189) with MSELoss(sum) * (1 / n), through mutils-style flattening."""
    from flpytorch_amd import harness
    A, B = DATA["data_A"], DATA["data_B"]
    m = harness.DenseModel(A, B, 16)
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Flatten(1), torch.nn.Linear(8, 32), torch.nn.ReLU(), torch.nn.Linear(32, 64),
                              torch.nn.ReLU(), torch.nn.Linear(64, 1), torch.nn.Sigmoid())
    x = torch.cat([p.detach().reshape(-1) for p in net.parameters()])
    xb, yb = torch.from_numpy(A[16:32]), torch.from_numpy(B[16:32])
    loss = torch.nn.MSELoss(reduction="sum")(net(xb), yb) * (1.0 / 16)
    loss.backward()
    g_ref = torch.cat([p.grad.reshape(-1) for p in net.parameters()])
    f, g = m.value_and_gradient(x, 1)
    assert f == (torch.zeros(1) + loss.detach()).item()
    assert torch.equal(g, g_ref)


def test_rejects_other_algorithms():
    from flpytorch_amd import harness
    m = harness.DenseModel(DATA["data_A"], DATA["data_B"], 16)
    with pytest.raises(ValueError):
        harness.Simulation("scaffold", "ident", m, np.zeros(m.D, np.float32), 4, 4, 1, 0.1, 1.0, device="cpu")
    with pytest.raises(ValueError):
        harness.Simulation("diana", "randk:10%", m, np.zeros(m.D, np.float32), 4, 4, 1, 0.1, 1.0, device="cpu",
                           wire=True)
    with pytest.raises(ValueError):
        harness.Simulation("diana", "randk:10%", m, np.zeros(m.D, np.float32), 4, 4, 1, 0.1, 1.0, device="cpu",
                           initialize_shifts_policy="random")


def test_find_recent_and_remove():
    """findRecentRecordAndRemoveFromHistory (algorithms.py:371-399): newest round first, the field
    is cleared once read, a round that sampled the client without the field ends the search."""
    from flpytorch_amd.harness import find_recent_and_remove
    H = {"history": {0: {"client_states": {1: {"client_state": {"hi": "a"}}, 2: {"client_state": {"hi": "b"}}}},
                     1: {"client_states": {1: {"client_state": {"hi": "c"}}}},
                     2: {"client_states": {2: {"client_state": {}}}}}}
    assert find_recent_and_remove(H, 1, "hi") == "c"
    assert H["history"][1]["client_states"][1]["client_state"]["hi"] is None
    assert find_recent_and_remove(H, 1, "hi") is None
    assert find_recent_and_remove(H, 2, "hi") is None          # round 2 sampled client 2 without "hi"
    assert find_recent_and_remove(H, 3, "hi") is None


def test_ef21_first_round_samples_every_client():
    sim = oracle_simulation("ef21_randk10_p2")
    sim.run_round(0)
    assert list(sim.H["history"][0]["client_states"]) == list(range(META["ef21_randk10_p2"]["num_clients"]))
    assert sim.H["request_use_full_list_of_clients"] is False
    sim.run_round(1)
    assert list(sim.H["history"][1]["client_states"]) == [int(c) for c in sim.sampled[1]]


@pytest.mark.parametrize("name", [n for n in RUN_NAMES if META[n]["algorithm"] == "marina"])
def test_marina_server_draws_follow_the_stream(name):
    """MARINA's serverGlobalStateUpdate draws np_random.random() after every round (algorithms.py:571):
    the harness's draws equal the reference run's, and each round's clients took the full-gradient
    branch exactly when the previous draw was <= p = 1 / (1 + w)."""
    sim = oracle_simulation(name)
    draws = []
    for r in range(sim.rounds):
        prev = sim.H["test_ber_rv"]
        sim.run_round(r)
        draws.append(sim.H["test_ber_rv"])
        for st in sim.H["history"][r]["client_states"].values():
            cs = st["client_state"]
            assert cs["ck"] == (1 if prev <= cs["p"] else 0)
    assert draws == META[name]["test_ber_rv"]


def test_poisson_runs_include_an_empty_round():
    """The Poisson fixture exercises fl_funcs.py:17-29's empty sample: zero clients, zero gradient."""
    m = META["dcgd_randk10_poisson"]
    empty = [r for r, h in enumerate(m["history"]) if not h["clients"]]
    assert empty and all(m["history"][r]["grad_sgd_server_l2"] == 0.0 for r in empty)
    assert all(h["clients"] for h in META["fedavg_poisson_no_empty"]["history"])
