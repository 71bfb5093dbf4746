#!/usr/bin/env python3
"""Generate the round-harness fixtures (tests/golden/harness.npz + harness.json) from the REAL
reference.

Test infrastructure only: runs in the development container where /root/reference is mounted;
the GPU box receives only the fixtures.  It drives ``fl_pytorch/run.py`` like make_golden.py
(same throwaway stubs for the packages the image lacks) and records what a harness needs to
replay a run without the reference:

* the synthetic client data the run trained on — ``ArificialDataset`` (data_preprocess/
  artificial_dataset.py:12-125), drawn from the experiment's ``np_random`` seeded with
  ``--manual-init-seed`` and SVD-conditioned; captured from the train set the run built
  (client c owns rows [c*S, (c+1)*S), artificial_dataset.py:178-186);
* the starting point x0 (``H['x0']``, algorithms.py:2000-2001) and the iterate after every
  round's global step (model_funcs.py:605);
* per round: the sampled clients in Buffer order (= the insertion order of
  ``H['history'][r]['client_states']``, algorithms.py:2193-2203), each client's
  ``approximate_f_value`` list and ``send_scalars_to_master``, and the history scalars
  ``grad_sgd_server_l2`` / ``x_before_round`` / ``approximate_f_avg_value``
  (algorithms.py:2218-2223).

Runs: the four of make_golden.py (C1 = FedAvg + ident; DCGD with randk / qsgd / topk) plus
partial participation (2 of 4 clients per round) with 2 local steps, for DCGD randk and FedAvg;
DIANA (randk / qsgd, zero and full-gradient initial shifts) and EF21 (topk = contraction, randk =
unbiased: the 1 / (1 + w) multiplier) over enough rounds that clients come back to their stored
shifts.  For DIANA the server shift h after every round's serverGlobalStateUpdate is recorded too.
"""
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (stubs, COMMON, REF)

RUNS = dict(mg.RUNS)
RUNS.update({
    "dcgd_randk10_p2_li2": ["--algorithm", "dcgd", "--client-compressor", "randk:10%",
                            "--num-clients-per-round", "2", "-li", "2", "--rounds", "4"],
    "fedavg_p2_li2": ["--algorithm", "fedavg", "--client-compressor", "ident",
                      "--num-clients-per-round", "2", "-li", "2", "--rounds", "4"],
    "diana_randk10_p2_li2": ["--algorithm", "diana", "--client-compressor", "randk:10%",
                             "--num-clients-per-round", "2", "-li", "2", "--rounds", "5"],
    "diana_qsgd10_fullgrad": ["--algorithm", "diana", "--client-compressor", "qsgd:10",
                              "--initialize-shifts-policy", "full_gradient_at_start", "--rounds", "3"],
    "ef21_topk10_p2_li2": ["--algorithm", "ef21", "--client-compressor", "topk:10%",
                           "--num-clients-per-round", "2", "-li", "2", "--rounds", "5"],
    "ef21_randk10_p2": ["--algorithm", "ef21", "--client-compressor", "randk:10%",
                        "--num-clients-per-round", "2", "--rounds", "5"],
    # Poisson client sampling (fl_funcs.py:17-40): per round and client one uniform() draw; the
    # plain form allows empty rounds (serverGradient -> zeros, algorithms.py:2117-2118), the
    # no-empty form redraws the whole round until someone is sampled
    "dcgd_randk10_poisson": ["--algorithm", "dcgd", "--client-compressor", "randk:10%",
                             "--client-sampling-type", "poisson", "--client-sampling-poisson", "0.3",
                             "--rounds", "8"],
    "fedavg_poisson_no_empty": ["--algorithm", "fedavg", "--client-compressor", "ident",
                                "--client-sampling-type", "poisson-no-empty", "--client-sampling-poisson", "0.3",
                                "--rounds", "8"],
    # MARINA (algorithms.py:480-573): the server's np_random.random() after every round (571)
    # decides full gradients vs g_prev + C(grad - grad_prev) for the next round
    "marina_randk10_li2": ["--algorithm", "marina", "--client-compressor", "randk:10%", "-li", "2",
                           "--rounds", "8"],
    "marina_qsgd10_p2_li2": ["--algorithm", "marina", "--client-compressor", "qsgd:10", "-li", "2",
                             "--num-clients-per-round", "2", "--rounds", "8"],
})


def main():
    tmp = tempfile.mkdtemp(prefix="flstubs_")
    mg._write_stubs(tmp)
    sys.path.insert(0, tmp)
    sys.path.insert(0, os.path.join(mg.REF, "utils"))
    sys.path.insert(0, mg.REF)
    sys.dont_write_bytecode = True
    scratch = tempfile.mkdtemp(prefix="flharness_")
    work = os.path.join(scratch, "a", "b")
    os.makedirs(work)
    os.chdir(work)
    import run as refrun                                  # reference modules, imported read-only
    from utils import algorithms, execution_context
    from models import mutils
    from data_preprocess import artificial_dataset

    # the iterate after every round's global step (the model holds it when serverGlobalStateUpdate
    # runs, model_funcs.py:605-607); x0 from the start hook (run.py prunes tensors from H at the end)
    iterates, starts, shifts, ber = [], [], [], []
    orig_sgsu = algorithms.serverGlobalStateUpdate

    def sgsu_wrap(clients_responses, model, *a, **k):
        iterates.append(mutils.get_params(model).detach().cpu().numpy().copy())
        Hn = orig_sgsu(clients_responses, model, *a, **k)
        if "test_ber_rv" in Hn:
            ber.append(Hn["test_ber_rv"])                                # MARINA's server draw
        if Hn["algorithm"] == "diana":
            shifts.append(Hn["h"].detach().cpu().numpy().copy())         # h after h += alpha m
        return Hn
    algorithms.serverGlobalStateUpdate = sgsu_wrap
    execution_context.simulation_start_fn = lambda H: starts.append(H["x0"].detach().cpu().numpy().copy())

    captured = []
    orig_init = artificial_dataset.ArificialDataset.__init__

    def init_wrap(self, exec_ctx, args, train=None, *a, **k):
        orig_init(self, exec_ctx, args, train, *a, **k)
        if train is None or train:
            captured.append((self.data.numpy().copy(), self.targets.numpy().copy(), self.n_client_samples))
    artificial_dataset.ArificialDataset.__init__ = init_wrap

    arrays, meta = {}, {}
    for name, extra in RUNS.items():
        captured.clear()
        iterates.clear()
        starts.clear()
        shifts.clear()
        ber.clear()
        result = {}
        execution_context.simulation_finish_fn = lambda H, _r=result: _r.update(H=H)
        refrun.runSimulation(mg.COMMON + extra + ["--run-id", name])
        H = result["H"]
        A, B, S = captured[0]
        if "data_A" in arrays:
            assert np.array_equal(arrays["data_A"], A) and np.array_equal(arrays["data_B"], B)
        arrays["data_A"], arrays["data_B"] = A, B
        arrays[f"{name}_x0"] = starts[0]
        arrays[f"{name}_iterates"] = np.stack(iterates)            # x after each round's global step
        if shifts:
            arrays[f"{name}_server_shift"] = np.stack(shifts)
        hist = H["history"]
        rounds = []
        for r in sorted(hist):
            cs = hist[r]["client_states"]
            order = list(cs.keys())
            rounds.append({
                "clients": [int(c) for c in order],
                "approximate_f_value": [[float(v) for v in cs[c]["client_state"]["approximate_f_value"]] for c in order],
                "send_scalars_to_master": [float(cs[c]["client_state"]["stats"]["send_scalars_to_master"]) for c in order],
                "grad_sgd_server_l2": float(hist[r]["grad_sgd_server_l2"]),
                "x_before_round": float(hist[r]["x_before_round"]),
                "approximate_f_avg_value": float(hist[r]["approximate_f_avg_value"]),
            })
        args = H["args"]
        meta[name] = {
            "argv": mg.COMMON + extra,
            "algorithm": args.algorithm, "client_compressor": args.client_compressor,
            "num_clients": int(H["total_clients"]), "clients_per_round": int(args.num_clients_per_round),
            "rounds": int(args.rounds), "local_iters": int(args.number_of_local_iters),
            "local_lr": float(args.local_lr), "global_lr": float(args.global_lr),
            "manual_runtime_seed": int(args.manual_runtime_seed), "samples_per_client": int(S),
            "D": int(H["D"]), "history": rounds,
            "initialize_shifts_policy": args.initialize_shifts_policy,
            "client_sampling_type": args.client_sampling_type,
            "client_sampling_poisson": float(args.client_sampling_poisson),
            "test_ber_rv": [float(v) for v in ber],
        }
        print(name, [r["grad_sgd_server_l2"] for r in rounds])
    np.savez_compressed(os.path.join(HERE, "harness.npz"), **arrays)
    with open(os.path.join(HERE, "harness.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
