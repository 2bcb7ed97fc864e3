"""Merge tools/pmc.sh summaries into profiles/pmc_kernels.json, the file
bench.py reads for roofline.traffic and roofline.valu_frac.

Per kernel: HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes;
the x2 is the gfx950 FETCH_SIZE correction of MI355X_MICROARCH.md section
HBM/rocprofv3), VALU / SALU / LDS instructions per launch and waves. The file
records the hash of the device code it was collected on (bench.code_object_hash:
the .hip_fatbin of the built libgsm.so); bench.py ignores it once the device
code changes, so stale counters never reach a bench line.

The fused rollout kernel ("roll") runs ROLL_STEPS steps per launch (env,
default 100: a 100-step graph); its entry is normalised to one step, so that
bench.py compares it with the launch time per step.

Usage: python tools/pmc_traffic.py OUT_JSON [KINDS@]KEY_PREFIX=SUMMARY_DIR ...
  e.g. h:navigation:N24:B8192=gpurun_out/pmc_h  (keys: step:navigation:N24:B8192, emit:...)
       lag@h:navigation:N24:B8192=gpurun_out/pmc_h_lag  (only the lagged step kernel)
       roll>rollbuf@b:navigation:N24:B8192=...  (the rollout kernel, stored as rollbuf:navigation:...)
"""
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "gs-marl_amd"))
from bench import code_object_hash  # noqa: E402

out_path = sys.argv[1]
h = code_object_hash()
res = json.load(open(out_path)) if os.path.exists(out_path) else {}
if res.get("code_object_hash") != h:   # entries from other builds are dropped, not mixed
    res = {}
res.update(code_object_hash=h, collected=time.strftime("%Y-%m-%d %H:%M:%S"))
ent = res.setdefault("entries", {})
for spec in sys.argv[2:]:
    key, d = spec.split("=", 1)
    kinds = None
    rename = {}
    if "@" in key:
        k0, key = key.split("@", 1)
        kinds = set()
        for kk in k0.split("+"):   # "roll>rollbuf": kernel roll stored under the name rollbuf
            src, _, dst = kk.partition(">")
            kinds.add(src)
            if dst:
                rename[src] = dst
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
        e = dict(hbm_bytes_per_launch=round(rd + wr), read_bytes_corrected=round(rd), write_bytes=round(wr),
                 fetch_size_kib=c["FETCH_SIZE"], write_size_kib=c["WRITE_SIZE"], dispatches=v["dispatches"],
                 source=d)
        PER_LAUNCH = (("SQ_INSTS_VALU", "valu_insts_per_launch"), ("SQ_INSTS_SALU", "salu_insts_per_launch"),
                      ("SQ_INSTS_LDS", "lds_insts_per_launch"), ("SQ_WAVE_CYCLES", "wave_quad_cycles_per_launch"),
                      ("SQ_ACTIVE_INST_ANY", "active_inst_any_quad_cycles_per_launch"),
                      ("SQ_WAIT_ANY", "wait_any_quad_cycles_per_launch"),
                      ("SQ_WAIT_INST_ANY", "wait_inst_any_quad_cycles_per_launch"),
                      ("GRBM_GUI_ACTIVE", "grbm_gui_active_per_launch"))
        for cn, k in PER_LAUNCH + (("SQ_WAVES", "waves"),):
            if cn in c:
                e[k] = c[cn]
        if kern == "roll":   # per step of the launch
            n = int(os.environ.get("ROLL_STEPS", "100"))
            for k in ("hbm_bytes_per_launch", "read_bytes_corrected", "write_bytes") + tuple(k for _, k in PER_LAUNCH):
                if k in e:
                    e[k] = round(e[k] / n, 1)
            e["per"] = f"step (counters of one {n}-step launch / {n})"
        ent[f"{rename.get(kern, kern)}:{key.split(':', 1)[1]}"] = e
json.dump(res, open(out_path, "w"), indent=1, sort_keys=True)
print(json.dumps(res, indent=1))
