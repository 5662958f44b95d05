import sys, time, os
sys.path.insert(0, '/root/repo'); os.chdir('/root/repo')
import numpy as np, torch
from apf_quadruped_amd import plans
import bench
plan = plans.standard_plan('c1'); plan.compile()
dev = torch.device('cuda', 0)
host = bench.make_shard(plan, plans.SEED + 1, 0, 1024)
vals = {k: torch.from_numpy(v).to(dev) for k, v in host.items()}
out = plan.alloc_outputs(1024, device=dev)
best = torch.zeros(2, dtype=torch.float64, device=dev)
s = torch.cuda.current_stream()
go = plan.launcher(vals, out, 1024, stream=s, best=best)
for _ in range(20): go()
torch.cuda.synchronize()
K = 400
t0 = time.perf_counter()
for _ in range(K): go()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print('no events: submit us/step %.2f, total us/step %.2f' % ((t1-t0)/K*1e6, (t2-t0)/K*1e6))
# graph of 20 steps
g = torch.cuda.CUDAGraph()
cs = torch.cuda.Stream()
cs.wait_stream(s)
with torch.cuda.stream(cs):
    go2 = plan.launcher(vals, out, 1024, stream=cs, best=best)
    go2(); torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=cs):
        for _ in range(20): go2()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(K // 20): g.replay()
torch.cuda.synchronize()
t2 = time.perf_counter()
print('graph x20: total us/step %.2f' % ((t2-t0)/K*1e6))
print('best', best.cpu().numpy())
