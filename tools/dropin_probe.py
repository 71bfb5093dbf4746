"""Where a lone compressVector's time goes: host submission cost per call vs device time per call.

  host_us        : perf_counter over R calls without a sync (Python + ctypes + the library's launches)
  device_us      : events around R calls, the calls submitted behind a long spin kernel so that the
                   host is ahead of the device (the device never waits for a submission)
  serial_us      : events around R calls submitted as the bench does (host and device race)

Usage: python3 tools/dropin_probe.py [--spec topk:1%] [--d 10000000] [--reps 200]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spec", default="topk:1%")
    ap.add_argument("--d", type=int, default=10_000_000)
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--spin-ms", type=float, default=60.0)
    ap.add_argument("--compat", action="store_true", help="dithering: the caller's float64 uniforms (as bench --dropin)")
    a = ap.parse_args()
    from flpytorch_amd import aggregation as ag
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    rows = torch.randn(a.n, a.d, generator=torch.Generator(device=dev).manual_seed(9), device=dev)
    comps = [ag.initCompressor(a.spec, a.d) for _ in range(a.n)]
    if any(c.compressorType in (ag.CompressorType.STANDARD_DITHERING_FP32,) for c in comps):
        for i, c in enumerate(comps):
            if a.compat:
                c.testp = torch.rand(a.d, dtype=torch.float64, device=dev)
            else:
                c.device_rng = (7, i)
    for i in range(a.n):
        comps[i].compressVector(rows[i])
    torch.cuda.synchronize()

    def calls():
        for r in range(a.reps):
            i = r % a.n
            comps[i].compressVector(rows[i])

    res = {"spec": a.spec, "d": a.d, "reps": a.reps, "compat": a.compat}
    t0 = time.perf_counter()
    calls()
    res["host_us"] = round((time.perf_counter() - t0) / a.reps * 1e6, 2)
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    e[0].record()
    calls()
    e[1].record()
    e[1].synchronize()
    res["serial_us"] = round(e[0].elapsed_time(e[1]) / a.reps * 1e3, 2)
    # behind a spin kernel: calibrate cycles for ~spin_ms
    torch.cuda.synchronize()
    cyc = 1_000_000
    e[0].record(); torch.cuda._sleep(cyc); e[1].record(); e[1].synchronize()
    per_ms = cyc / max(e[0].elapsed_time(e[1]), 1e-3)
    e[0].record()
    torch.cuda._sleep(int(per_ms * a.spin_ms))
    e[1].record()
    t0 = time.perf_counter()
    calls()
    sub_ms = (time.perf_counter() - t0) * 1e3
    e[2].record()
    e[2].synchronize()
    spin = e[0].elapsed_time(e[1])
    res["device_us"] = round(e[1].elapsed_time(e[2]) / a.reps * 1e3, 2)
    res["spin_ms"] = round(spin, 2)
    res["submit_ms"] = round(sub_ms, 2)
    res["host_ahead"] = bool(sub_ms < spin)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
