"""Where the spread of a headline rollout launch comes from: per-wave marks of
tools/stamps_h_timeline.py (saved with STAMPS_NPZ) grouped by XCD, by the
workgroup's dispatch rank on its CU, and by the time its state had loaded.

Marks (µs from the first wave's entry): 0 entry, 1 state loaded, 4 step K-1
published, 8 final state stored. Prints JSON: per group the mean / max of each
mark, and the correlation of a wave's load time with its last publish.

Usage: python tools/stamps_h_spread.py gpurun_out/st1/h20.npz"""
import json
import sys

import numpy as np


def main(path):
    z = np.load(path)
    q, hw = z["stamps"].astype(np.int64), z["hw"].astype(np.int64)
    t0 = q[:, 0].min()
    us = {n: (q[:, i] - t0) / 100.0 for n, i in (("entry", 0), ("loaded", 1), ("published_last", 4),
                                                  ("stored", 8))}
    xcc = (hw >> 32) & 7
    cu = xcc << 8 | ((hw >> 13) & 7) << 5 | ((hw >> 12) & 1) << 4 | ((hw >> 8) & 15)
    B = len(q)
    wg = np.arange(B) // 4
    rank = np.zeros(B, dtype=np.int64)
    for c in np.unique(cu):
        sel = np.nonzero(cu == c)[0]
        for r, g in enumerate(np.unique(wg[sel])):
            rank[sel[wg[sel] == g]] = r
    out = {}

    def stats(mask):
        return {n: [round(float(v[mask].mean()), 2), round(float(v[mask].max()), 2)] for n, v in us.items()}

    out["by_xcc"] = {int(x): stats(xcc == x) for x in np.unique(xcc)}
    out["by_rank"] = {int(r): stats(rank == r) for r in np.unique(rank)}
    # per CU: its latest publish against its latest load
    cus = np.unique(cu)
    ld = np.array([us["loaded"][cu == c].max() for c in cus])
    pb = np.array([us["published_last"][cu == c].max() for c in cus])
    out["cu_corr_loaded_vs_published_last"] = round(float(np.corrcoef(ld, pb)[0, 1]), 3)
    out["cu_published_last_pct"] = {p: round(float(np.percentile(pb, p)), 2) for p in (0, 10, 50, 90, 100)}
    slow = cus[np.argsort(pb)[-8:]]
    out["slowest_cus"] = [{"cu": int(c), "xcc": int(c >> 8), "loaded_max": round(float(us["loaded"][cu == c].max()), 2),
                           "published_last_max": round(float(us["published_last"][cu == c].max()), 2)}
                          for c in slow]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
