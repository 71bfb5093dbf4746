#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the REAL reference.

Test infrastructure only. Runs in the development container, where the reference
is mounted read-only at /root/reference; it is never run on the GPU box (the
fixtures it writes are committed and travel instead).

What it captures
----------------
1. ``codecs.npz``   — per compressor spec / D / input distribution: the inputs, the
   patterns drawn by ``Compressor.generateCompressPattern`` from a seeded
   ``np.random.RandomState`` (fl_pytorch/utils/compressors.py:196-216), the dense
   ``compressVector`` outputs (compressors.py:218-371), the wire-size stats
   (compressors.py:25-38, 223-224, 367-368) and the constants the algorithms read
   (compressors.py:64-194).  Clients are drawn in the order the reference uses
   inside one round: pattern draws, then ``randint(2**31)`` for the client seed
   (algorithms.py:2015-2069, seed at 2055).
2. ``rng.npz``      — numpy legacy MT19937 stream values for the calls the reference
   makes: ``choice(D, K, replace=False)`` (compressors.py:206), ``rand(D)`` (208-212),
   ``random()`` (204), ``randint(2**31)`` (algorithms.py:2055) and the client
   sampling ``choice(n, m, replace=False)`` (fl_funcs.py:15).
3. ``runs.npz`` + ``runs.json`` — ``fl_pytorch/run.py`` driven end to end (config C1 of
   BASELINE.json plus DCGD with randk / qsgd), with the ``serverGradient`` inputs and
   outputs captured per round (algorithms.py:1748-1770, 1810-1832) and the per-round
   history scalars (algorithms.py:2218-2223).

The third-party modules the reference imports but this image lacks (coloredlogs,
wandb, h5py, torchvision) are replaced by throwaway stubs written to a temporary
directory at run time (never into /root/reference or the repository); torchvision's
download helper is stubbed to RAISE so no fetch can happen.  Reference sources are
imported, never copied.
"""
import json
import os
import sys
import tempfile
import textwrap

import numpy as np

REF = "/root/reference/fl_pytorch"
HERE = os.path.dirname(os.path.abspath(__file__))


def _write_stubs(root):
    files = {
        "coloredlogs/__init__.py": "def install(*a, **k):\n    pass\n",
        "wandb/__init__.py": textwrap.dedent("""
            def login(*a, **k):
                raise ValueError('wandb stub: offline')
            def init(*a, **k):
                raise ValueError('wandb stub: offline')
            def log(*a, **k):
                pass
        """),
        "h5py/__init__.py": "",
        "torchvision/__init__.py": "from . import models, transforms, datasets\n",
        "torchvision/models/__init__.py": textwrap.dedent("""
            def _nope(*a, **k):
                raise RuntimeError('torchvision stub')
            resnet18 = resnet34 = resnet50 = _nope
        """),
        "torchvision/transforms/__init__.py": textwrap.dedent("""
            class _T:
                def __init__(self, *a, **k):
                    pass
                def __call__(self, x):
                    return x
            Compose = ToTensor = Normalize = RandomCrop = RandomHorizontalFlip = _T
        """),
        "torchvision/datasets/__init__.py": textwrap.dedent("""
            from . import utils
            class CIFAR10:
                def __init__(self, *a, **k):
                    raise RuntimeError('torchvision stub: no datasets offline')
            CIFAR100 = CIFAR10
        """),
        "torchvision/datasets/utils.py": textwrap.dedent("""
            def download_url(*a, **k):
                raise RuntimeError('torchvision stub: network access refused')
        """),
    }
    for rel, body in files.items():
        p = os.path.join(root, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(body)


# ----------------------------------------------------------------------------------------------
# 1. codec fixtures
# ----------------------------------------------------------------------------------------------
DISTS = ["normal", "heavy", "zeros", "ties", "powers"]


def make_input(dist, D, client, base_seed=2024):
    """Client rows. Drawn from a generator that does NOT touch the shared pattern stream."""
    g = np.random.default_rng([base_seed, client, D, DISTS.index(dist)])
    if dist == "normal":
        x = g.standard_normal(D)
    elif dist == "heavy":
        x = g.standard_normal(D) * 10.0 ** g.uniform(-3, 3, D)
    elif dist == "zeros":
        x = g.standard_normal(D)
        x[g.random(D) < 0.3] = 0.0
    elif dist == "ties":
        # few distinct magnitudes, both signs: exercises TopK ties and exact level hits
        x = g.integers(-4, 5, D).astype(np.float64) * 0.25
    elif dist == "powers":
        # exact powers of two and level boundaries (natural / dithering edge cases)
        x = np.ldexp(1.0, g.integers(-20, 20, D)) * g.choice([-1.0, 1.0], D)
    else:
        raise ValueError(dist)
    return x.astype(np.float32)


CODEC_CASES = [
    # (spec, D, dist, n_clients)
    ("ident", 1000, "normal", 2),
    ("randk:1%", 1000, "normal", 3),
    ("randk:1%", 2465, "normal", 3),      # D/K inexact (98.6)
    ("randk:10%", 4099, "heavy", 3),
    ("randk:37", 1000, "normal", 2),
    ("randk:100%", 257, "normal", 2),
    ("randk:1%", 1, "normal", 2),
    ("randk:1%", 65536, "normal", 2),
    ("bernulli:0.5", 1000, "normal", 4),
    ("bernulli:0.2", 1000, "normal", 4),
    ("natural", 4099, "normal", 3),
    ("natural", 4099, "heavy", 2),
    ("natural", 1000, "zeros", 2),
    ("natural", 1000, "powers", 2),
    ("qsgd:127", 4099, "normal", 3),
    ("qsgd:127", 4099, "heavy", 2),
    ("qsgd:127", 1000, "zeros", 2),
    ("qsgd:127", 1000, "ties", 2),
    ("qsgd:127", 65536, "normal", 2),
    ("qsgd:10", 1000, "normal", 2),
    ("qsgd:1", 1000, "normal", 2),
    ("std.dithering:10:2", 1000, "normal", 2),
    ("std.dithering:8", 1000, "normal", 2),
    ("std.dithering:4:inf", 1000, "ties", 2),
    ("std.dithering:7:1", 1000, "normal", 2),
    ("terngrad", 1000, "normal", 2),
    ("nat.dithering:10:2", 1000, "normal", 2),
    ("nat.dithering:4", 1000, "normal", 2),
    ("topk:1%", 4099, "normal", 3),
    ("topk:1%", 65536, "heavy", 2),
    ("topk:50%", 8, "normal", 1),
    ("topk:3", 1000, "normal", 2),
    ("topk:10%", 1000, "zeros", 2),
    ("topk:10%", 1000, "ties", 2),
    ("topk:100%", 100, "normal", 1),
    ("topk:1%", 1, "normal", 1),
]


def codec_fixtures(compressors, torch):
    out = {}
    meta = []
    for ci, (spec, D, dist, n_clients) in enumerate(CODEC_CASES):
        rs = np.random.RandomState(123 + ci)
        pre = f"c{ci:02d}_"
        rows, outs, pats, seeds, stats, pnorms = [], [], [], [], [], []
        info = None
        for c in range(n_clients):
            comp = compressors.initCompressor(spec, D)
            comp.generateCompressPattern(rs, "cpu", c, None)
            seeds.append(rs.randint(2 ** 31))  # algorithms.py:2055
            x = make_input(dist, D, c)
            xt = torch.from_numpy(x.copy())
            y = comp.compressVector(xt)
            rows.append(x)
            outs.append(y.numpy().astype(np.float32).copy())
            t = comp.compressorType
            if t == 3:
                pats.append(comp.S.numpy().astype(np.int64))
            elif t in (4, 5, 6):
                pats.append(comp.testp.numpy().astype(np.float64))
            elif t == 2:
                pats.append(np.array([comp.testp], dtype=np.float64))
            else:
                pats.append(np.zeros(0))
            if t in (5, 6):
                pnorms.append(float(torch.norm(xt, p=comp.p)))
            else:
                pnorms.append(float("nan"))
            stats.append([comp.total_input_components, comp.really_need_to_send_components,
                          comp.last_input_advance, comp.last_need_to_send_advance])
            if info is None:
                info = {
                    "spec": spec, "D": D, "dist": dist, "n_clients": n_clients, "seed": 123 + ci,
                    "type": t, "fullName": comp.fullName(),
                    "K": getattr(comp, "K", None),
                    "w": getattr(comp, "w", None),
                    "alpha": getattr(comp, "alpha", None),
                    "s": getattr(comp, "s", None),
                    "p": (None if not hasattr(comp, "p") else (float(comp.p) if t in (5, 6) else comp.p)),
                    "P": getattr(comp, "P", None),
                    "isUnbiased": comp.isUnbiasedCompressor(),
                    "isContraction": comp.isContractionCompressor(),
                }
                if hasattr(comp, "levelsValues"):
                    out[pre + "levels"] = comp.levelsValues.cpu().numpy().astype(np.float32)
        info["client_seeds"] = [int(s) for s in seeds]
        info["after_draws"] = [int(v) for v in rs.randint(2 ** 31, size=4)]
        out[pre + "x"] = np.stack(rows)
        out[pre + "out"] = np.stack(outs)
        out[pre + "stats"] = np.array(stats, dtype=np.float64)
        out[pre + "pnorm"] = np.array(pnorms, dtype=np.float64)
        # Patterns: keep RandK index sets (small) and lazy draws; dithering uniforms are
        # regenerated by the oracle's MT19937 and pinned through rng.npz + the outputs.
        if info["type"] in (2, 3):
            for c, p in enumerate(pats):
                out[pre + f"pat{c}"] = p
        elif info["type"] in (4, 5, 6) and D <= 1000:
            out[pre + "pat0"] = pats[0]
        meta.append(info)
    return out, meta


# ----------------------------------------------------------------------------------------------
# 2. RNG stream fixtures (the numpy legacy calls the reference makes)
# ----------------------------------------------------------------------------------------------
def rng_fixtures():
    out = {}
    meta = []
    cases = [
        ("choice", 0, (10, 10)), ("choice", 123, (1000, 10)), ("choice", 7, (2465, 25)),
        ("choice", 2 ** 31 - 1, (100000, 1000)), ("choice", 5, (1, 1)), ("choice", 11, (4099, 4099)),
        ("choice", 42, (3, 2)),
        ("rand", 0, (17,)), ("rand", 123, (1000,)), ("rand", 4294967295, (5,)),
        ("random", 9, (3,)),
        ("randint31", 123, (16,)),
        ("seq", 123, ()),   # interleaved sequence like a DCGD randk round
    ]
    for i, (kind, seed, args) in enumerate(cases):
        rs = np.random.RandomState(seed)
        key = f"r{i:02d}"
        if kind == "choice":
            out[key] = rs.choice(args[0], args[1], replace=False).astype(np.int64)
        elif kind == "rand":
            out[key] = rs.rand(args[0])
        elif kind == "random":
            out[key] = np.array([rs.random() for _ in range(args[0])])
        elif kind == "randint31":
            out[key] = np.array([rs.randint(2 ** 31) for _ in range(args[0])], dtype=np.int64)
        elif kind == "seq":
            # fl_funcs.py:15 sampling for 2 rounds, then per client choice(D,K) + randint(2**31)
            vals = []
            for _ in range(2):
                vals.extend(rs.choice(10, 4, replace=False).tolist())
            for _ in range(4):
                vals.extend(rs.choice(2465, 247, replace=False).tolist())
                vals.append(rs.randint(2 ** 31))
            vals.extend(rs.rand(3).view(np.int64).tolist())
            out[key] = np.array(vals, dtype=np.int64)
        st = rs.get_state()
        meta.append({"kind": kind, "seed": seed, "args": list(args), "end_pos": int(st[2])})
        out[key + "_endkey"] = np.asarray(st[1][:8], dtype=np.uint32)
    return out, meta


# ----------------------------------------------------------------------------------------------
# 3. run.py end-to-end captures (config C1 + DCGD)
# ----------------------------------------------------------------------------------------------
RUNS = {
    "c1_fedavg_ident": ["--algorithm", "fedavg", "--client-compressor", "ident"],
    "dcgd_randk10": ["--algorithm", "dcgd", "--client-compressor", "randk:10%"],
    "dcgd_qsgd10": ["--algorithm", "dcgd", "--client-compressor", "qsgd:10"],
    "dcgd_topk5": ["--algorithm", "dcgd", "--client-compressor", "topk:5%"],
}
COMMON = ("--rounds 3 --num-clients-per-round 4 --dataset generated_for_quadratic_minimization "
          "--dataset-generation-spec clients:4,samples_per_client:16,variables:8,homogeneous:0,l:1.0,mu:0.1 "
          "--model dense --loss mse --metric loss --algorithm-options internal_sgd:full-gradient "
          "--gpu -1 --deterministic -li 1 --run-local-steps --local-lr 0.1 --global-lr 1.0 "
          "--eval-every 1 --manual-init-seed 123 --manual-runtime-seed 456").split()


def run_fixtures(torch):
    scratch = tempfile.mkdtemp(prefix="flgolden_")
    work = os.path.join(scratch, "a", "b")
    os.makedirs(work)
    cwd = os.getcwd()
    os.chdir(work)
    try:
        import run as refrun                     # reference module, imported read-only
        from utils import algorithms, compressors, execution_context
        arrays, scalars = {}, {}
        pats = []
        orig_gen = compressors.Compressor.generateCompressPattern

        def gen_wrap(self, rndgen, device, clientId, H):
            orig_gen(self, rndgen, device, clientId, H)
            if clientId >= 0 and self.compressorType == 3:
                pats.append(self.S.numpy().copy())
        compressors.Compressor.generateCompressPattern = gen_wrap

        for name, extra in RUNS.items():
            pats.clear()
            cls = algorithms.getImplClassForAlgo(extra[1])
            orig = cls.serverGradient
            captured = []

            def sg(clients_responses, clients, model, params_current, H, _orig=orig, _cap=captured):
                rows = []
                for i in range(clients):
                    clients_responses.waitForItem()
                    rows.append(clients_responses.get(i)["model"].detach().cpu().numpy().copy())
                for i in range(clients):          # hand the semaphore back to the original
                    clients_responses.item_is_ready.release()
                res = _orig(clients_responses, clients, model, params_current, H)
                _cap.append((params_current.detach().cpu().numpy().copy(), np.stack(rows),
                             res.detach().cpu().numpy().copy()))
                return res
            cls.serverGradient = staticmethod(sg)
            result = {}
            execution_context.simulation_finish_fn = lambda H, _r=result: _r.update(H=H)
            refrun.runSimulation(COMMON + extra + ["--run-id", name])
            cls.serverGradient = staticmethod(orig)
            H = result["H"]
            hist = H["history"]
            scalars[name] = {
                "rounds": len(captured),
                "D": int(H["D"]),
                "grad_sgd_server_l2": [float(hist[r]["grad_sgd_server_l2"]) for r in sorted(hist)],
                "x_before_round": [float(hist[r]["x_before_round"]) for r in sorted(hist)],
                "approximate_f_avg_value": [float(hist[r]["approximate_f_avg_value"]) for r in sorted(hist)],
                "send_scalars_to_master": [[float(hist[r]["client_states"][c]["client_state"]["stats"]["send_scalars_to_master"])
                                            for c in sorted(hist[r]["client_states"])] for r in sorted(hist)],
                "global_lr": 1.0,
            }
            for r, (x, rows, gs) in enumerate(captured):
                arrays[f"{name}_r{r}_x"] = x
                arrays[f"{name}_r{r}_models"] = rows
                arrays[f"{name}_r{r}_gs"] = gs
            if pats:
                arrays[f"{name}_patterns"] = np.stack(pats).astype(np.int64)
        return arrays, scalars
    finally:
        os.chdir(cwd)


def main():
    tmp = tempfile.mkdtemp(prefix="flstubs_")
    _write_stubs(tmp)
    sys.path.insert(0, tmp)
    sys.path.insert(0, os.path.join(REF, "utils"))
    sys.path.insert(0, REF)
    sys.dont_write_bytecode = True
    import torch
    import compressors  # /root/reference/fl_pytorch/utils/compressors.py

    a, m = codec_fixtures(compressors, torch)
    np.savez_compressed(os.path.join(HERE, "codecs.npz"), **a)
    with open(os.path.join(HERE, "codecs.json"), "w") as f:
        json.dump(m, f, indent=1)
    print("codecs:", len(m), "cases")

    a, m = rng_fixtures()
    np.savez_compressed(os.path.join(HERE, "rng.npz"), **a)
    with open(os.path.join(HERE, "rng.json"), "w") as f:
        json.dump(m, f, indent=1)
    print("rng:", len(m), "cases")

    if "--no-runs" not in sys.argv:
        a, s = run_fixtures(torch)
        np.savez_compressed(os.path.join(HERE, "runs.npz"), **a)
        with open(os.path.join(HERE, "runs.json"), "w") as f:
            json.dump(s, f, indent=1)
        print("runs:", s)


if __name__ == "__main__":
    main()
