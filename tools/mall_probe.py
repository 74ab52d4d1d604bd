"""Does a buffer written and read back soon after come from the MALL
(Infinity Cache) rather than HBM?  For buffer sizes around the MALL
capacity: time x.sum() right after writing x, and after writing a 4 GB
buffer in between (x evicted).  Diagnostic for the X round trip of the
data pass -> moment pass; not part of the product."""
import json
import torch

dev = torch.device("cuda:0")
big = torch.empty(4 << 30 >> 3, dtype=torch.float64, device=dev)
out = {}
for mb in (32, 64, 128, 192, 256, 384, 512, 1024, 4096):
    n = (mb << 20) >> 3
    x = torch.empty(n, dtype=torch.float64, device=dev)
    st = torch.cuda.Event(enable_timing=True)
    en = torch.cuda.Event(enable_timing=True)
    res = {}
    for mode in ("hot", "cold"):
        ts = []
        for _ in range(5):
            x.fill_(1.0)
            if mode == "cold":
                big.fill_(2.0)
            torch.cuda.synchronize()
            st.record()
            s = x.sum()
            en.record()
            torch.cuda.synchronize()
            ts.append(st.elapsed_time(en))
        t = min(ts)
        res[mode] = {"ms": round(t, 4), "gbs": round(n * 8 / t / 1e6, 1)}
    # write bandwidth into a buffer just read (fill only)
    ts = []
    for _ in range(5):
        torch.cuda.synchronize()
        st.record()
        x.fill_(3.0)
        en.record()
        torch.cuda.synchronize()
        ts.append(st.elapsed_time(en))
    res["fill_gbs"] = round(n * 8 / min(ts) / 1e6, 1)
    out[mb] = res
    print(mb, res, flush=True)
    del x
print(json.dumps(out))
