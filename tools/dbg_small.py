import sys, os
sys.path.insert(0, os.getcwd())
import torch, parallel_kd_tree_amd as pk
from parallel_kd_tree_amd import ops
dev = torch.device("cuda:0")
for n in [17, 33, 60, 64, 65, 100, 129, 200, 256, 257, 300, 1000]:
    x = pk.generate_problem(n, 3, n)
    b = ops.GpuTreeBuilder(n, 3)
    tp, ti = b.build(x.to(dev))
    torch.cuda.synchronize()
    det = b.read_error_detail()
    cp, ci = ops.build_cpu(x, None, "exact", 0, 1)
    same = torch.equal(ti.cpu(), ci)
    bad = (ti.cpu() != ci).nonzero().flatten()[:10].tolist()
    print(n, "same", same, "err", [hex(v) for v in det], "first bad slots", bad, flush=True)
