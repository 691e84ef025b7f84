"""Arrival skew of the resident MGS sweep: per pass and block, the wall clock (100 MHz) at the end of
the block's streaming and after its hand-off completes, dumped by nkb_mgs_res (NK_RES_TSTAMP).
Usage: NK_RES_TSTAMP=/tmp/ts.bin python tools/kbench_res.py --ks 30 --rvs 89 --reps 1 &&
       python tools/res_skew.py /tmp/ts.bin 30"""
import sys

import numpy as np

ts = np.fromfile(sys.argv[1], dtype=np.uint64).astype(np.float64)
k = int(sys.argv[2])
G = ts.size // (2 * k)
ts = ts.reshape(k, G, 2) * 10e-3  # 100 MHz ticks -> us
end, done = ts[..., 0], ts[..., 1]
pass_len = np.diff(np.median(done, axis=1))
print(f"{G} blocks, {k} passes; median pass {np.median(pass_len):.2f} us")
skew = end.max(1) - end.min(1)
lat = done.min(1) - end.max(1)
spread = done.max(1) - done.min(1)
print(f"arrival skew (last - first block end): median {np.median(skew):.2f} us, max {skew.max():.2f}")
print(f"hand-off latency (last end -> first done): median {np.median(lat):.2f} us")
print(f"completion spread (first -> last done): median {np.median(spread):.2f} us")
late = (end - np.median(end, axis=1, keepdims=True))[1:].mean(0)  # mean lateness per block
print("mean lateness by blockIdx % 8 (us):", " ".join(f"{late[np.arange(G) % 8 == x].mean():+.2f}" for x in range(8)))
order = np.argsort(late)
print("earliest blocks:", order[:8].tolist(), "latest blocks:", order[-8:].tolist())
print("lateness quantiles (us): " + " ".join(f"{q}%:{np.percentile(late, q):+.2f}" for q in (0, 10, 50, 90, 100)))
# is lateness persistent? correlation of the lateness of consecutive passes
e = end - np.median(end, axis=1, keepdims=True)
cors = [np.corrcoef(e[t], e[t + 1])[0, 1] for t in range(1, k - 1)]
print(f"pass-to-pass lateness correlation: median {np.median(cors):.2f}")
