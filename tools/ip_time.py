import sys, time, torch
sys.path.insert(0, '/root/repo')
from opticalflowfromdepth_amd import forward_warp_flow, ops, synth
dev = torch.device('cuda:0')
seeds = [12345 + i for i in range(64)]
obj, flow, depth = synth.stage_one_batch(seeds, 768, 1024, dev)
out, valid, coll = forward_warp_flow(obj, flow, depth)
rgb = (out[:, 0:3] * valid).contiguous()
print('hole frac', float((valid == 0).float().mean()), flush=True)
for i in range(3):
    torch.cuda.synchronize(); t = time.perf_counter()
    r = ops.inpaint(rgb, valid, coll)
    torch.cuda.synchronize(); print('inpaint 64 imgs ms', (time.perf_counter() - t) * 1e3, flush=True)
