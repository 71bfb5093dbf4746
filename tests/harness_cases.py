"""Shared setup of the round-harness tests: the reference runs captured by
tests/golden/make_golden_harness.py (harness.json / harness.npz) replayed through
flpytorch_amd.harness.Simulation."""
import numpy as np

from tests.golden_io import load

META, DATA = load("harness")
RUN_NAMES = sorted(META)


def simulation(name, device, **kw):
    from flpytorch_amd import harness
    m = META[name]
    model = harness.DenseModel(DATA["data_A"], DATA["data_B"], m["samples_per_client"])
    assert model.D == m["D"]
    return harness.Simulation(m["algorithm"], m["client_compressor"], model, DATA[f"{name}_x0"], m["num_clients"],
                              m["clients_per_round"], m["rounds"], m["local_lr"], m["global_lr"],
                              local_iters=m["local_iters"], runtime_seed=m["manual_runtime_seed"], device=device,
                              initialize_shifts_policy=m.get("initialize_shifts_policy", "zero"),
                              sampling=m.get("client_sampling_type", "uniform"),
                              poisson_p=m.get("client_sampling_poisson"), **kw)


def check_server_shift(name, rounds_h, rtol=1e-5, atol=1e-7):
    """DIANA: the server shift h after each round's serverGlobalStateUpdate (algorithms.py:1424-1428)
    against the reference run's (``rounds_h``: the harness's h per round, collected by the test)."""
    want = DATA[f"{name}_server_shift"]
    assert len(rounds_h) == len(want)
    for r, (got, w) in enumerate(zip(rounds_h, want)):
        np.testing.assert_allclose(got, w, rtol=rtol, atol=atol, err_msg=f"{name} h after round {r}")


def check_history(name, H, rel=1e-6):
    """Per round: the sampled clients in Buffer order, each client's f values and wire counts, and the
    history scalars of serverGlobalStateUpdate (algorithms.py:2218-2223) within `rel` of the
    reference's."""
    want = META[name]["history"]
    assert len(H["history"]) == len(want)
    for r, w in enumerate(want):
        got = H["history"][r]
        assert list(got["client_states"]) == w["clients"], (name, r)
        for c, fv, snd in zip(w["clients"], w["approximate_f_value"], w["send_scalars_to_master"]):
            cs = got["client_states"][c]["client_state"]
            np.testing.assert_allclose(cs["approximate_f_value"], fv, rtol=rel, err_msg=f"{name} r{r} c{c} f")
            assert cs["stats"]["send_scalars_to_master"] == snd, (name, r, c)
        for k in ("grad_sgd_server_l2", "x_before_round", "approximate_f_avg_value"):
            if np.isnan(w[k]):                           # an empty round: no f values (np.mean of [])
                assert np.isnan(got[k]), (name, r, k, got[k])
                continue
            assert abs(got[k] - w[k]) <= rel * abs(w[k]), (name, r, k, got[k], w[k])
