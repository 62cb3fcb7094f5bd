"""Values of one gradient: ours vs fp32 oracle vs float64 oracle (debug aid)."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.chdir(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import test_models_gpu as T  # noqa: E402
from tests.golden import fixtures as FX  # noqa: E402

case = FX.case_by_name(sys.argv[1])
pname = sys.argv[2]
ora, ours = T.build(case, "fp32")
ins, eps = FX.inputs_fn(case)(0)
ora64 = copy.deepcopy(ora).double()
T.run_oracle_step(case, ora64, [t.double() for t in ins], eps.double())
T.run_oracle_step(case, ora, ins, eps)
T.run_ours_step(case, ours, ins, eps)
g_m = dict(ours.named_parameters())[pname].grad.cpu().double()
g_o = dict(ora.named_parameters())[pname].grad.double()
g_d = dict(ora64.named_parameters())[pname].grad
print("torch threads", torch.get_num_threads(), "mkldnn", torch.backends.mkldnn.is_available())
print("ours ", g_m.reshape(-1)[:6].tolist(), float(g_m.norm()))
print("o32  ", g_o.reshape(-1)[:6].tolist(), float(g_o.norm()))
print("o64  ", g_d.reshape(-1)[:6].tolist(), float(g_d.norm()))
print("rel ours-o64", T.rel(g_m, g_d), "rel o32-o64", T.rel(g_o, g_d), "rel ours-o32", T.rel(g_m, g_o))
d = (g_m - g_d).reshape(-1).abs()
idx = torch.argsort(d, descending=True)[:12]
print("worst idx", idx.tolist())
print("ours", g_m.reshape(-1)[idx].tolist())
print("o64 ", g_d.reshape(-1)[idx].tolist())
print("n entries rel err > 1e-3:", int(((d / g_d.reshape(-1).abs().clamp_min(1e-3)) > 1e-3).sum()), "of", d.numel())
