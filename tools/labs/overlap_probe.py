import os, sys, json
import numpy as np, torch
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tools')
import synth
from lambdafs_amd import HipReedSolomonCode, device
k, p, L, S = 10, 4, 1 << 20, 1024
code = HipReedSolomonCode(k, p, device=0)
st = torch.zeros((S, k + p, L), dtype=torch.uint8, device="cuda")
synth.fill_data_rows(torch, st, 3, 0, k, p)
to_read = sorted(code.locationsToReadForDecode([p]))
ntr = [x for x in range(k + p) if x not in to_read]
D = code.decodeMatrix([p], ntr)[:, to_read]
out = torch.empty((S, 1, L), dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
def seq():
    device.encode_stripes(code, st)
    device.apply_rows(code, D, [st[:, l, :] for l in to_read], [out[:, 0, :]])
def ovl(nchunks):
    c = S // nchunks
    evs = []
    for i in range(nchunks):
        with torch.cuda.stream(s1):
            device.encode_stripes(code, st[i*c:(i+1)*c])
            e = torch.cuda.Event(); e.record(s1)
        s2.wait_event(e)
        with torch.cuda.stream(s2):
            device.apply_rows(code, D, [st[i*c:(i+1)*c, l, :] for l in to_read], [out[i*c:(i+1)*c, 0, :]])
    torch.cuda.current_stream().wait_stream(s1); torch.cuda.current_stream().wait_stream(s2)
def timed(fn, n=20):
    fn(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n): fn()
    b.record(); b.synchronize()
    return a.elapsed_time(b) / n
for rep in range(3):
    r = {"seq": timed(seq)}
    for nc in (2, 4, 8):
        r[f"ovl{nc}"] = timed(lambda: ovl(nc))
    ok = torch.equal(out[:, 0], st[:, p])
    print(json.dumps({k2: round(v, 4) for k2, v in r.items()} | {"ok": ok}), flush=True)
