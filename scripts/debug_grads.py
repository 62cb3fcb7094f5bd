"""Per-parameter gradient error of one fixture case vs the oracle (debug aid): python scripts/debug_grads.py CASE [dtype]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.chdir(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import test_models_gpu as T  # noqa: E402
from tests.golden import fixtures as FX  # noqa: E402

case = FX.case_by_name(sys.argv[1])
ora, ours = T.build(case, sys.argv[2] if len(sys.argv) > 2 else "fp32")
ins, eps = FX.inputs_fn(case)(0)
masks, flat = (T.simple_masks(case, case["B"]) if case["kind"] == "simple" else (None, None))
o_out, o_loss = T.run_oracle_step(case, ora, ins, eps, masks)
m_out, m_loss = T.run_ours_step(case, ours, ins, eps, flat)
for i, (a, b) in enumerate(zip(m_out, o_out)):
    if a is not None and b is not None:
        print(f"out{i} rel {T.rel(a.detach(), b.detach()):.3e}")
mp = dict(ours.named_parameters())
for n, p in ora.named_parameters():
    print(f"{n:40s} rel {T.rel(mp[n].grad, p.grad):.3e}  bias->BN {T._bias_feeds_bn(ora, n)}")
for (n, bo), (_, bm) in zip(ora.named_buffers(), ours.named_buffers()):
    if bo.dtype.is_floating_point:
        print(f"buf {n:36s} rel {T.rel(bm, bo):.3e}")
