"""Histogram of the scalar-path instructions (tools/isa_cost.py classes) in one
loop of a kernel's assembly (diagnostic). Usage: python tools/isa_hist.py FILE.s KERNEL LOOP_LABEL [class]"""
import re
import sys
from collections import Counter

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from isa_cost import classify  # noqa: E402

path, kname, loop = sys.argv[1:4]
want = sys.argv[4] if len(sys.argv) > 4 else "scalar"
lines = open(path).read().splitlines()
st = next(i for i, l in enumerate(lines) if l.startswith(kname + ":"))
hdr = loop.replace(".LBB", "BB")
c = Counter()
inloop = False
for l in lines[st + 1:]:
    if l.startswith(".Lfunc_end"):
        break
    m = re.match(r"^(\.LBB\d+_\d+):(.*)", l) or re.match(r"^; %bb\.(\d+):(.*)", l)
    if m:
        inloop = f"Header={hdr} " in m.group(2) or m.group(1) == loop
        continue
    t = l.strip()
    if not t or t.startswith((";", ".")):
        continue
    p = t.split(None, 1)
    mn, ops = p[0], (p[1].split(";")[0] if len(p) > 1 else "")
    if inloop and classify(mn, ops) == want:
        c[re.sub(r"_e(32|64)$", "", mn)] += 1
for k, v in c.most_common(45):
    print(v, k)
