"""Static issue-cost census of a kernel's gfx950 assembly (diagnostic).

Counts, per loop and for the whole kernel, the instructions by the issue
resource they draw on (measured by tools/probe_issue.hip):

  scalar  SALU, and every VALU instruction that reads or writes an SGPR or
          VCC (v_readlane, v_writelane, v_readfirstlane, a compare into an
          SGPR pair or VCC, v_cndmask / v_addc on a lane mask, any SGPR
          operand): together at most ~0.96 per CU and cycle, shared by the
          CU's four SIMDs
  valu    VALU with only VGPR / inline-constant operands: ~0.45 per SIMD and
          cycle
  lds     ds_*: ~0.45 per CU and cycle (ds_read_b64)
  vmem, smem, branch, other (s_nop, s_waitcnt, barriers)

Usage: python tools/isa_cost.py FILE.s KERNEL_SUBSTRING
(e.g. build with: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off
 --cuda-device-only -S -Iinclude -Igs-marl_amd/csrc gs-marl_amd/csrc/gsm_ragged_kernels.hip -o ragged.s)
"""
import re
import sys
from collections import Counter, defaultdict

OTHER_S = ("s_nop", "s_waitcnt", "s_barrier", "s_sleep", "s_setprio", "s_endpgm", "s_sendmsg", "s_trap",
           "s_memtime", "s_memrealtime", "s_dcache", "s_icache", "s_inst_prefetch", "s_clause", "s_delay_alu",
           "s_sethalt", "s_ttracedata")
SGPR_OPERAND = re.compile(r"(?<![\w\]])(s\[\d+(:\d+)?\]|s\d+|vcc(_lo|_hi)?|ttmp\d+|m0)(?![\w])")
IMPLICIT_VCC = re.compile(r"^v_(cmp\w*_e32|cmpx\w*|cndmask_b32_e32|addc_co_u32_e32|subb_co_u32_e32|subbrev_co_u32_e32|"
                          r"add_co_u32_e32|sub_co_u32_e32|subrev_co_u32_e32|div_scale\w*|div_fmas\w*|"
                          r"readfirstlane\w*|readlane\w*|writelane\w*)")


def classify(mn, ops):
    if mn.startswith("s_"):
        if mn.startswith(("s_load", "s_buffer_load", "s_store", "s_buffer_store", "s_atomic", "s_scratch")):
            return "smem"
        if mn.startswith(("s_branch", "s_cbranch")):
            return "branch"
        if mn.startswith(OTHER_S):
            return "other"
        return "scalar"
    if mn.startswith("v_"):
        if IMPLICIT_VCC.match(mn) or SGPR_OPERAND.search(ops):
            return "scalar"
        return "valu"
    if mn.startswith("ds_"):
        return "lds"
    if mn.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def main(path, kname):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^[\w.$]+:", l) and kname in l and not l.startswith("."))
    blocks = defaultdict(Counter)   # block label -> counts
    loop_of = {}                     # block -> innermost loop header
    order = []
    cur = "entry"
    order.append(cur)
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\d+_\d+):(.*)", l)
        m2 = re.match(r"^; %bb\.(\d+):(.*)", l)
        if m or m2:
            cur = m.group(1) if m else f"%bb.{m2.group(1)}"
            rest = m.group(2) if m else m2.group(2)
            order.append(cur)
            h = re.search(r"Header=BB(\d+_\d+) Depth=(\d+)", rest)
            if "Loop Header" in rest:
                loop_of[cur] = (cur, int(re.search(r"Depth=(\d+)", rest).group(1)))
            elif h:
                loop_of[cur] = (".LBB" + h.group(1), int(h.group(2)))
            continue
        t = l.strip()
        if t.startswith(";") and "Loop Header" in t and blocks[cur].total() == 0:
            # the loop annotation on the line after the label ("Parent Loop ...")
            loop_of[cur] = (cur, int(re.search(r"Depth=(\d+)", t).group(1)))
            continue
        if not t or t.startswith((";", ".", "//")):
            continue
        parts = t.split(None, 1)
        mn = parts[0]
        ops = parts[1].split(";")[0] if len(parts) > 1 else ""
        blocks[cur][classify(mn, ops)] += 1
    cats = ("scalar", "valu", "lds", "vmem", "smem", "branch", "other")
    tot = Counter()
    for b in order:
        tot.update(blocks[b])
    print(f"{kname}: static totals " + " ".join(f"{c}={tot[c]}" for c in cats))
    loops = defaultdict(Counter)
    depth = {}
    for b in order:
        if b in loop_of:
            hdr, d = loop_of[b]
            loops[hdr].update(blocks[b])
            depth[hdr] = d
    for hdr in sorted(loops, key=lambda h: order.index(h) if h in order else 0):
        c = loops[hdr]
        print(f"  loop {hdr} depth {depth[hdr]}: " + " ".join(f"{k}={c[k]}" for k in cats))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
