"""Debug: run one trellis fixture row (index given) through the GPU kernel."""
import os, sys
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "aom-av1-lavish_amd"))
import numpy as np, torch
import _oracle as O
import lavish_dsp as L
from lavish_dsp import txb
F = dict(np.load(os.path.join(ROOT, "tests/golden/fix_trellis.npz")))
J = {n: i for i, n in enumerate(F["row_fields"])}
costs = txb.CoeffCosts(txb.coeff_costs_blob(F["coeff_costs"], F["eob_costs"]))
want = int(sys.argv[1])
for r in F["rows"]:
    g = lambda k: int(r[J[k]])
    if g("index") != want: continue
    s = g("tx_size"); n = L.max_eob(s); i = want
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    tc, qc, dq = dev(F["coeff"][i:i+1, :n]), dev(F["qcoeff_in"][i:i+1, :n]), dev(F["dqcoeff_in"][i:i+1, :n])
    eob = dev(np.array([g("eob_in")], np.int16))
    ctx = dev(np.array([[g("txb_skip_ctx"), g("dc_sign_ctx")]], np.int32))
    dqv = O.quant_arrays(O.build_quant(g("bd"), g("qindex")))["dequant"]
    rate, ec = txb.optimize_b_batch(costs, tc, qc, dq, eob, s, g("tx_type"), g("bd"), g("rdmult"), dqv,
                                    g("plane"), g("is_inter"), g("sharpness"), ctx, g("tx_type_cost"))
    torch.cuda.synchronize()
    print("GPU rate", int(rate[0]), "want", g("rate"), "eob", int(eob[0]), g("eob"), flush=True)
    print("GPU qc", qc.cpu().numpy()[0].tolist()); print("REF qc", F["qcoeff"][i][:n].tolist())
