"""Debug aid (GPU box): run the MARINA qsgd reference replay through the oracle-backed harness and
the product harness side by side, round by round, and report the first client whose model differs
and how its compressed step differs (oracle compressVector vs the product's fused shift codec)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tests.harness_cases import META, simulation  # noqa: E402
from tests.test_harness import (OracleCompressorDouble, oracle_marina_step,  # noqa: E402
                                oracle_server_gradient)
from flpytorch_amd import aggregation as ag  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "marina_qsgd10_p2_li2"
steps = []


def product_step(comp, g, g_old, g_prev):
    out = ag.marinaStep(comp, g.cuda(), g_old.cuda(), g_prev.cuda()).cpu()
    o = OracleCompressorDouble(comp.fullName() if False else META[name]["client_compressor"], g.numel())
    o.o.testp = comp.testp.cpu().numpy() if torch.is_tensor(comp.testp) else comp.testp
    want = g_prev + o.compressVector(g - g_old)
    diff = (out != want).sum().item()
    if diff:
        d = (g - g_old).numpy()
        pn_o = float(o.o.norm(d))
        pn_g = torch.empty(1, device="cuda")
        comp._encode_gpu((g - g_old).cuda(), pnorm_out=pn_g)
        steps.append((diff, pn_o, float(pn_g.item()), float(np.abs(d).max()), int((d == 0).sum()), d.size))
    return out


sim_o = simulation(name, "cpu", init_compressor=OracleCompressorDouble, server_gradient=oracle_server_gradient,
                   marina_step=oracle_marina_step)
sim_g = simulation(name, "cpu", marina_step=product_step)
for r in range(sim_o.rounds):
    sim_o.run_round(r)
    sim_g.run_round(r)
    a, b = sim_o.H["history"][r], sim_g.H["history"][r]
    print(r, a["grad_sgd_server_l2"], b["grad_sgd_server_l2"], "ber", sim_o.H["test_ber_rv"], sim_g.H["test_ber_rv"],
          "mismatching steps", steps[-3:] if steps else None, flush=True)
    steps.clear()
