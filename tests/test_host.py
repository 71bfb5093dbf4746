"""CPU tests of the product's host side: the C ABI exports, the compat-mode numpy stream and the
Compressor protocol constants (no GPU compute is called here)."""
import math
import re

import numpy as np
import pytest
import torch

from flpytorch_amd import _lib
from flpytorch_amd import aggregation as ag
from oracle import codecs as oc
from oracle.rng import OracleRandomState
from tests.golden_io import load

HEADER = __import__("os").path.join(__import__("os").path.dirname(__file__), "..", "include", "flcodec.h")


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    declared = set(re.findall(r"\b(flc_[a-z0-9_]+)\s*\(", open(HEADER).read()))
    assert declared == set(_lib.EXPORTS)
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.flc_version() == _lib.ABI_VERSION == 104


def test_library_build_id_matches_tree():
    """Provenance: the shipped .so reports the digest of the sources it was built from, and it is
    this tree's (smoke() and bench.py refuse a stale library the same way)."""
    assert _lib.build_id() == _lib.source_hash()
    assert _lib.check_provenance() == _lib.source_hash()


def test_library_is_gfx950():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


@pytest.mark.parametrize("seed", [0, 1, 123, 2 ** 32 - 1])
def test_stream_matches_numpy_and_oracle(seed):
    rs_np = np.random.RandomState(seed)
    rs_ag = np.random.RandomState(seed)
    rs_or = OracleRandomState(seed)
    for (n, k) in [(1, 1), (10, 10), (1000, 10), (2465, 247), (70000, 700)]:
        a = ag.stream_choice(rs_ag, n, k)
        np.testing.assert_array_equal(a, rs_np.choice(n, k, replace=False))
        np.testing.assert_array_equal(a, rs_or.choice(n, k))
        assert int(ag.stream_randint31(rs_ag)[0]) == rs_np.randint(2 ** 31) == rs_or.randint31()
    np.testing.assert_array_equal(ag.stream_rand(rs_ag, 1001), rs_np.rand(1001))
    assert ag.stream_random(rs_ag) == rs_np.random()
    # the RandomState object itself continues the same stream afterwards
    np.testing.assert_array_equal(rs_ag.randint(0, 1000, 50), rs_np.randint(0, 1000, 50))


@pytest.mark.parametrize("odd_words", [1, 3, 623])
def test_stream_rand_from_an_odd_position(odd_words):
    """rand(D) after an odd number of 32-bit draws (each client's randint(2**31),
    algorithms.py:2055, flips the parity): bit-exact, and on the block-copy path (fast)."""
    import time
    rs_np, rs_ag = np.random.RandomState(77), np.random.RandomState(77)
    for _ in range(odd_words):
        assert int(ag.stream_randint31(rs_ag)[0]) == rs_np.randint(2 ** 31)
    assert rs_ag.get_state()[2] % 2 == 1
    for n in (1, 2, 623, 624, 625, 1249):
        np.testing.assert_array_equal(ag.stream_rand(rs_ag, n), rs_np.rand(n))
    assert rs_ag.get_state()[2] % 2 == 1          # rand draws words in pairs: still odd
    n = 4_000_000
    t0 = time.perf_counter()
    got = ag.stream_rand(rs_ag, n)
    dt = time.perf_counter() - t0
    np.testing.assert_array_equal(got, rs_np.rand(n))
    assert rs_ag.get_state()[2] == rs_np.get_state()[2]
    assert dt < 0.5, f"rand({n}) from an odd position took {dt:.2f} s (scalar path?)"


def test_stream_rejects_other_generators():
    with pytest.raises((TypeError, AttributeError)):
        ag.stream_choice(np.random.default_rng(0), 10, 3)


CODEC_META, _ = load("codecs")


@pytest.mark.parametrize("m", CODEC_META, ids=[f"{m['spec']}-{m['D']}" for m in CODEC_META])
def test_compressor_constants_match_reference(m):
    c = ag.initCompressor(m["spec"], m["D"])
    assert c.compressorType == m["type"]
    assert c.fullName() == m["fullName"]
    assert getattr(c, "K", None) == m["K"]
    assert getattr(c, "w", None) == m["w"]
    assert getattr(c, "alpha", None) == m["alpha"]
    assert c.isUnbiasedCompressor() == m["isUnbiased"]
    assert c.isContractionCompressor() == m["isContraction"]
    if m["type"] in (5, 6):
        assert c.s == m["s"] and float(c.p) == m["p"]
        np.testing.assert_array_equal(c.levelsValues.numpy(), oc.OracleCompressor(m["spec"], m["D"]).levels)


def test_unknown_spec_raises_assertion():
    with pytest.raises(AssertionError):
        ag.initCompressor("gzip:9", 10)


def test_rank_k_constants():
    c = ag.initCompressor("rank_k:100%", 8)
    assert (c.A, c.B, c.K) == (2, 4, 8) and c.alpha == 4.0   # A = first divisor >= int(sqrt(D))


def test_generate_pattern_advances_stream_like_reference():
    rs_a, rs_b = np.random.RandomState(5), np.random.RandomState(5)
    for spec, draw in [("randk:10%", lambda r: r.choice(100, 10, replace=False)),
                       ("qsgd:4", lambda r: r.rand(100)), ("bernulli:0.3", lambda r: r.random()),
                       ("natural", lambda r: r.rand(100)), ("topk:5", lambda r: None), ("ident", lambda r: None)]:
        c = ag.initCompressor(spec, 100)
        c.generateCompressPattern(rs_a, "cpu", 0, None)
        ref = draw(rs_b)
        if spec.startswith("randk"):
            np.testing.assert_array_equal(c.S.numpy(), ref)
        elif spec.startswith(("qsgd", "natural")):
            np.testing.assert_array_equal(c.testp.numpy(), ref)
        elif spec.startswith("bernulli"):
            assert c.testp == ref
    assert rs_a.randint(2 ** 31) == rs_b.randint(2 ** 31)


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU behaviour")
def test_compute_without_gpu_fails_loudly():
    c = ag.initCompressor("topk:1", 10)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        c.compressVector(torch.ones(10))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ag.reduce_rows(torch.ones(4), [torch.ones(4)])
    # identity stays an alias, like the reference (compressors.py:228): no compute involved
    x = torch.ones(3)
    assert ag.initCompressor("ident", 3).compressVector(x) is x


def test_device_rng_host_mirror():
    lib = _lib.load()
    for d, k in [(1, 1), (7, 3), (1000, 10), (4097, 4097), (1 << 20, 10486), (4096 * 5 + 7, 20000)]:
        idx = np.empty(k, dtype=np.int64)
        assert lib.flc_device_randk_indices(42, 3, d, k, idx.ctypes.data) == 0
        assert idx.min() >= 0 and idx.max() < d and np.unique(idx).size == k
    u = np.array([lib.flc_device_uniform(42, 3, j) for j in range(20000)])
    assert u.min() >= 0.0 and u.max() < 1.0 and abs(u.mean() - 0.5) < 0.01
    assert math.isclose(np.var(u), 1 / 12, rel_tol=0.03)


@pytest.mark.parametrize("seed,client,d,k", [(42, 3, 1, 1), (42, 3, 7, 3), (1, 0, 4096, 4096), (42, 3, 4097, 4097),
                                             (5, 9, 1_000_000, 10_000), (7, 2, 4096 * 3 + 5, 100),
                                             (2**63 + 5, 10**9, 10_000_000, 100_000), (3, 4, 65536, 1)])
def test_device_randk_oracle_restatement(seed, client, d, k):
    """oracle/devrng.py restates the device RandK sampler (randk_tree.hpp: chunk counts of the row
    permutation's first K images + chunk permutations) in numpy; it equals the library's host
    mirror exactly."""
    from oracle import devrng
    lib = _lib.load()
    want = np.empty(k, dtype=np.int64)
    assert lib.flc_device_randk_indices(seed, client, d, k, want.ctypes.data) == 0
    got = devrng.randk_indices(seed, client, d, k)
    assert np.array_equal(got, want)
    assert np.unique(got).size == k and got.min() >= 0 and got.max() < d
    assert devrng.randk_counts(seed, client, d, k).sum() == k


def test_device_randk_is_uniform():
    """Device RandK sets behave as uniform K-subsets: every element kept with probability K/D (the
    unbiasedness RandK's w = D/K - 1 assumes) and chunk counts with the multivariate
    hypergeometric mean and variance."""
    lib = _lib.load()
    d, k, clients = 4096 * 6 + 1000, 500, 3000
    hits = np.zeros(d)
    counts = []
    for cl in range(clients):
        idx = np.empty(k, dtype=np.int64)
        assert lib.flc_device_randk_indices(77, cl, d, k, idx.ctypes.data) == 0
        hits[idx] += 1
        counts.append(np.bincount(idx // 4096, minlength=7))
    p = k / d
    # per-element frequency: binomial(clients, p) per element
    z = (hits - clients * p) / math.sqrt(clients * p * (1 - p))
    assert abs(z.mean()) < 0.05 and 0.9 < z.std() < 1.1
    counts = np.array(counts)
    for c in range(7):
        size = min(4096, d - c * 4096)
        q = size / d
        mean, var = k * q, k * q * (1 - q) * (d - k) / (d - 1)
        assert abs(counts[:, c].mean() - mean) < 4 * math.sqrt(var / clients)
        assert 0.85 < counts[:, c].var() / var < 1.15


def test_device_rng_oracle_restatement():
    """oracle/devrng.py (numpy) states the kernels' draw arithmetic independently; it equals the
    library's host mirror of the same generator (common.hpp dev_u32) on every index tried."""
    from oracle import devrng
    lib = _lib.load()
    for seed, client in [(42, 3), (0, 0), (2**63 + 5, 10**9), (20240607, 11)]:
        j = np.concatenate([np.arange(5000), [2**31 - 1, 2**31, 2**32 - 1, 123456789]]).astype(np.int64)
        got = devrng.dev_u32(seed, client, j.astype(np.uint32)).astype(np.float64) / 2**32
        ref = np.array([lib.flc_device_uniform(seed, client, int(v)) for v in j])
        assert np.array_equal(got, ref)
    # the top byte: one group hash serves the 4 elements of an aligned group, byte (j & 3) each
    u = devrng.dev_u32(7, 1, np.arange(1 << 16, dtype=np.uint32))
    top = (u >> np.uint32(24)).astype(np.int64)
    assert abs(top.mean() - 127.5) < 2.0 and np.unique(top).size == 256


@pytest.mark.parametrize("rk", [0x12345678, 0xDEADBEEF, 7])
def test_device_rng_group_hash_statistics(rk):
    """The group hash that supplies the draws' top bytes (common.hpp gmix over a keyed Weyl
    sequence): over 2^20 consecutive groups, no bit is biased, no pair of bits is correlated within
    a word or between words 1, 2, 64 or 1024 groups apart, and the 4 bytes of a group (4 elements'
    top bytes) and neighbouring groups' bytes are jointly uniform — each statistic within what
    independent uniform bits give (|z| < 5.5 over the ~5000 pairs, chi^2 / dof < 1.35)."""
    import math
    from oracle import devrng
    n = 1 << 20
    g = np.arange(n, dtype=np.uint32)
    h = devrng.grouphash(g, np.uint32(rk))
    bits = ((h[:, None] >> np.arange(32, dtype=np.uint32)) & np.uint32(1)).astype(np.float32) * 2 - 1
    assert np.abs(bits.mean(0)).max() * math.sqrt(n) < 5.5
    for lag in (0, 1, 2, 64, 1024):
        a, b = (bits, bits) if lag == 0 else (bits[:-lag], bits[lag:])
        c = (a.T @ b) / len(a)
        if lag == 0:
            np.fill_diagonal(c, 0)
        assert np.abs(c).max() * math.sqrt(len(a)) < 5.5, lag
    by = [((h >> np.uint32(8 * q)) & np.uint32(0xFF)).astype(np.int64) for q in range(4)]

    def chi2(cells, bins):
        cnt = np.bincount(cells, minlength=bins)
        e = len(cells) / bins
        return ((cnt - e) ** 2 / e).sum() / (bins - 1)
    assert max(chi2(b, 256) for b in by) < 1.35
    assert chi2((by[0] >> 6) * 64 + (by[1] >> 6) * 16 + (by[2] >> 6) * 4 + (by[3] >> 6), 256) < 1.35
    assert chi2((by[3][:-1] >> 4) * 16 + (by[0][1:] >> 4), 256) < 1.35


def test_c_client_of_the_abi(tmp_path):
    """include/flcodec.h compiles as C99 (-pedantic, no warnings) and a C program linked against
    libflcodec.so gets the same host-side answers as the Python binding (tests/c/abi_host.c)."""
    import os
    import shutil
    import subprocess
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    root = os.path.join(os.path.dirname(__file__), "..")
    libdir = os.path.dirname(_lib.LIB_PATH)
    exe = str(tmp_path / "abi_host")
    cc = subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-pedantic", "-Werror",
                         "-I" + os.path.join(root, "include"), os.path.join(root, "tests", "c", "abi_host.c"),
                         "-L" + libdir, "-lflcodec", "-Wl,-rpath," + libdir, "-o", exe],
                        capture_output=True, text=True)
    assert cc.returncode == 0, cc.stderr
    run = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert run.returncode == 0, run.stdout + run.stderr
    assert "OK" in run.stdout


def test_install_rebinds_every_shared_fold():
    """install() rebinds the reference classes whose serverGradient is the shared fold
    (algorithms.py: FedAvg, FedProx, MARINA, PP-MARINA, SCAFFOLD plain; DCGD, EF21, EF21PP with the
    master compressor; DIANA, COFIG, GradSkip, FRECON with their own tails) and restores them."""
    import types
    names = ["FedAvg", "FedProx", "MarinaAlgorithm", "MarinaAlgorithmPP", "SCAFFOLD", "DCGD", "EF21", "EF21PP",
             "DIANA", "COFIG", "GradSkip", "FRECON"]
    orig = {}
    algos = types.SimpleNamespace()
    for n in names:
        def sg(*a, _n=n):
            return _n
        orig[n] = sg
        setattr(algos, n, type(n, (), {"serverGradient": staticmethod(sg)}))
    comps = types.SimpleNamespace(initCompressor=lambda *a: "ref", Compressor=object)
    restore = ag.install(comps, algos)
    assert comps.initCompressor is ag.initCompressor
    want = {**{n: ag.serverGradientPlain for n in ag.PLAIN_FOLD}, **{n: ag.serverGradientMaster for n in ag.MASTER_FOLD},
            **ag.SHIFTED_FOLD}
    for n in names:
        fn = getattr(algos, n).serverGradient
        if n in want:
            assert fn is want[n], n
        elif n == "FRECON":
            assert fn is not orig[n] and "FRECON" in fn.__doc__
        else:
            assert fn is orig[n], n
    restore()
    for n in names:
        assert getattr(algos, n).serverGradient is orig[n]
    assert comps.initCompressor() == "ref"


def test_install_mapping_matches_the_reference_classes(tmp_path):
    """The class names install() rebinds are exactly the reference's algorithm classes that define a
    serverGradient (read from fl_pytorch/utils/algorithms.py itself, imported in a subprocess with
    the throwaway stubs of tests/golden/make_golden.py; skipped where the reference is absent)."""
    import json
    import os
    import subprocess
    import sys
    ref = "/root/reference/fl_pytorch"
    if not os.path.isdir(ref):
        pytest.skip("reference not mounted (GPU box / other hosts)")
    here = os.path.dirname(os.path.abspath(__file__))
    code = f"""
import json, sys, inspect
sys.path.insert(0, {os.path.join(here, 'golden')!r})
import make_golden
make_golden._write_stubs({str(tmp_path)!r})
sys.path.insert(0, {str(tmp_path)!r}); sys.path.insert(0, {ref + '/utils'!r}); sys.path.insert(0, {ref!r})
from utils import algorithms
names = sorted(n for n, c in inspect.getmembers(algorithms, inspect.isclass)
               if c.__module__ == algorithms.__name__ and 'serverGradient' in c.__dict__)
print(json.dumps(names))
"""
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       cwd=str(tmp_path), env={**os.environ, "PYTHONDONTWRITEBYTECODE": "1"})
    assert r.returncode == 0, r.stderr[-2000:]
    ref_names = set(json.loads(r.stdout.strip().splitlines()[-1]))
    ours = set(ag.PLAIN_FOLD) | set(ag.MASTER_FOLD) | set(ag.SHIFTED_FOLD) | {"FRECON"}
    assert ours == ref_names, (sorted(ours ^ ref_names))


@pytest.mark.parametrize("spec", ["topk:1%", "randk:1%", "qsgd:127", "qsgd:4", "ident"])
def test_torch_cpu_baseline_matches_oracle(spec):
    """oracle/torch_cpu.py (the reference's torch calls, timed as bench.py's cpu_baseline) computes
    what the numpy oracle computes: same numpy-stream patterns, bit-equal outputs (dithering given
    torch's own CPU norm), and the fold equals server_gradient."""
    import torch
    from oracle import codecs as oc
    from oracle.rng import OracleRandomState
    from oracle.torch_cpu import TorchCpuCodec, fold
    d = 20011
    g = np.random.default_rng(3).standard_normal((3, d)).astype(np.float32)
    rs_t, rs_o = np.random.RandomState(77), OracleRandomState(77)
    outs = []
    for i in range(3):
        t = TorchCpuCodec(spec, d)
        t.generate(rs_t)
        o = oc.OracleCompressor(spec, d)
        o.generate(rs_o)
        x = torch.from_numpy(g[i])
        got = t.compress(x).numpy()
        pn = float(torch.norm(x, p=2)) if spec.startswith("qsgd") else None
        want = o.compress(g[i], pnorm=pn) if pn is not None else o.compress(g[i])
        assert np.array_equal(got.view(np.uint32), np.asarray(want, np.float32).view(np.uint32))
        outs.append(got)
    x0 = np.zeros(d, np.float32)
    models = [x0 - e for e in outs]
    gs = fold(torch.from_numpy(x0), [torch.from_numpy(m) for m in models]).numpy()
    assert np.array_equal(gs.view(np.uint32), oc.server_gradient(x0, models).view(np.uint32))


def test_torch_cpu_time_uplink_phases():
    from oracle.torch_cpu import time_uplink
    r = time_uplink(["randk:1%", "topk:1%", "qsgd:4"], 10007, budget_s=0.01)
    assert r["clients"] >= 2 and all(r[k] >= 0 for k in ("pattern_s", "compress_s", "fold_s"))


def test_torch_norm_oracle_vs_torch_on_this_host():
    """oracle/torch_norm.c restates torch.norm(x, p=2) for CPU fp32 tensors (compressors.py:272):
    bit-equal to torch itself here for lengths around the 8-lane accumulator and its tail, and
    mixed magnitudes.  (The GPU kernel flc_norm2_torch_cpu is checked against this restatement in
    tests/test_gpu_norm_torch.py; the reference's recorded norms pin both in
    tests/test_oracle_golden.py.)"""
    import ctypes

    import numpy as np
    import torch

    from oracle import rng
    # the restatement's 8 lanes are torch's AVX2 Vectorized<float>.  The norm kernel has
    # no AVX512 registration, so an AVX512 host (this container reports "AVX512") runs the same AVX2
    # kernel — this test pins that; a torch without AVX2 ("DEFAULT", non-x86) is unpinned
    cap = torch.backends.cpu.get_cpu_capability()
    if cap not in ("AVX2", "AVX512"):
        pytest.skip(f"torch's {cap} CPU kernels: the 8-lane (AVX2) restatement is unpinned here")
    rng._load()
    lib = ctypes.CDLL(rng._LIB_PATH)
    lib.orc_torch_norm2.restype = ctypes.c_float
    lib.orc_torch_norm2.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    g = np.random.default_rng(2025)
    for d in [1, 3, 7, 8, 9, 15, 16, 17, 100, 1001, 4099, 65543, 300_007]:
        for _ in range(3):
            x = (g.standard_normal(d) * 10.0 ** g.uniform(-3, 3, d)).astype(np.float32)
            want = np.float32(torch.norm(torch.from_numpy(x), p=2).item())
            got = np.float32(lib.orc_torch_norm2(x.ctypes.data, d))
            assert got.view(np.uint32) == want.view(np.uint32), (d, got, want)
