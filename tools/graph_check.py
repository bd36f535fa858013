import sys, importlib, numpy as np, torch
sys.path.insert(0, '.')
torch.cuda.is_available()
wg = importlib.import_module('wireguard-java_amd')
dev = torch.device('cuda', 0)
n, L = 4096, 1420
S = 1440
off = np.arange(n, dtype=np.uint64) * S
desc = wg.pack_desc(off, off, np.arange(n, dtype=np.uint64), np.full(n, L), np.zeros(n, np.int64))
eng = wg.Engine(0, key_slots=1)
eng.set_keys(0, bytes(range(32)))
d = torch.from_numpy(wg.desc_as_int64(desc)).to(dev)
pt = torch.randint(0, 256, (n * S,), dtype=torch.uint8, device=dev)
ct = torch.zeros_like(pt); back = torch.zeros_like(pt); st = torch.zeros(n, dtype=torch.int32, device=dev)
eng.duplex(d, pt, ct, L, d, ct, back, st, L, uniform=True, after_seal=True)
torch.cuda.synchronize()
ref = ct.clone()
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
with torch.cuda.graph(g):
    print('capturing on', torch.cuda.current_stream().cuda_stream, torch.cuda.is_current_stream_capturing())
    eng.duplex(d, pt, ct, L, d, ct, back, st, L, uniform=True, after_seal=True)
torch.cuda.synchronize()
ct.zero_(); back.zero_(); torch.cuda.synchronize()
g.replay(); torch.cuda.synchronize()
print('replay refilled ct:', bool(torch.equal(ct, ref)), 'back ok:', bool(torch.equal(back.view(n, S)[:, :L], pt.view(n, S)[:, :L])))
