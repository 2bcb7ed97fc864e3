"""Merge tools/pmc.sh summaries into profiles/pmc_traffic.json, the file
bench.py reads for roofline.traffic: HBM bytes per launch of each kernel =
2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes; the x2 is the gfx950 FETCH_SIZE
correction of MI355X_MICROARCH.md section HBM/rocprofv3).

Usage: python tools/pmc_traffic.py OUT_JSON [KINDS@]KEY_PREFIX=SUMMARY_DIR ...
  e.g. h:navigation:N24:B8192=gpurun_out/pmc_h  (keys: step:navigation:N24:B8192, emit:...)
       lag@h:navigation:N24:B8192=gpurun_out/pmc_h_lag  (only the lagged step kernel)
"""
import json
import os
import sys

out_path = sys.argv[1]
res = json.load(open(out_path)) if os.path.exists(out_path) else {}
for spec in sys.argv[2:]:
    key, d = spec.split("=", 1)
    kinds = None
    if "@" in key:
        k0, key = key.split("@", 1)
        kinds = set(k0.split("+"))
    txt = open(os.path.join(d, "summary.txt")).read()
    summ = json.loads(txt[txt.index("{"):])
    for kern, v in summ.items():
        if kinds is not None and kern not in kinds:
            continue
        c = v["counters"]
        if "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
            continue
        rd = 2 * c["FETCH_SIZE"] * 1024
        wr = c["WRITE_SIZE"] * 1024
        res[f"{kern}:{key.split(':', 1)[1]}"] = dict(
            hbm_bytes_per_launch=round(rd + wr), read_bytes_corrected=round(rd), write_bytes=round(wr),
            fetch_size_kib=c["FETCH_SIZE"], write_size_kib=c["WRITE_SIZE"], dispatches=v["dispatches"],
            source=d)
json.dump(res, open(out_path, "w"), indent=1, sort_keys=True)
print(json.dumps(res, indent=1))
