"""Instruction histogram of a kernel's hottest loop (the largest basic-block cycle) in a .s file."""
import re
import sys
from collections import Counter

path, kname = sys.argv[1], sys.argv[2]
s = open(path).read()
starts = [(m.start(), m.group(1)) for m in re.finditer(r"^(_Z\w+):[ ;]", s, re.M)]
for i, (pos, name) in enumerate(starts):
    if kname not in name:
        continue
    end = starts[i + 1][0] if i + 1 < len(starts) else len(s)
    lines = s[pos:end].splitlines()
    # locate loop: a backward branch s_cbranch*/s_branch to an earlier label
    labels = {l.split(":")[0]: j for j, l in enumerate(lines) if re.match(r"^\.LBB\w+:", l)}
    best = None
    for j, l in enumerate(lines):
        m = re.match(r"\s+s_(cbranch_\w+|branch)\s+(\.LBB\w+)", l)
        if m and m.group(2) in labels and labels[m.group(2)] < j:
            span = j - labels[m.group(2)]
            if best is None or span > best[1] - best[0]:
                best = (labels[m.group(2)], j)
    body = [l.split()[0] for l in lines[best[0]:best[1] + 1] if l.startswith("\t") and not l.startswith("\t.") and not l.startswith("\t;")]
    c = Counter(body)
    print(name, "loop instrs", len(body))
    groups = Counter()
    for op, n in c.items():
        if op.startswith("v_") and "f64" in op: g = "valu_f64"
        elif op.startswith(("v_rcp", "v_sqrt", "v_rsq", "v_exp", "v_log")): g = "valu_trans"
        elif op.startswith("v_readlane") or op.startswith("v_writelane"): g = "lane_spill"
        elif op.startswith("v_"): g = "valu_other"
        elif op.startswith("s_waitcnt"): g = "waitcnt"
        elif op.startswith("s_"): g = "salu/branch"
        elif op.startswith("ds_"): g = "lds"
        elif op.startswith(("global_", "buffer_", "flat_")): g = "vmem"
        elif op.startswith("scratch_"): g = "scratch"
        else: g = "other"
        groups[g] += n
    print(dict(groups))
    print(c.most_common(45))
    break
