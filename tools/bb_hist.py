"""Largest basic blocks of a kernel in a .s file, with their instruction mix (hot-path triage)."""
import re
import sys
from collections import Counter

path, kname = sys.argv[1], sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 3
s = open(path).read()
i = s.index(kname)
i = s.index(":", i)
j = s.index(".Lfunc_end", i)
blocks, cur, name = [], [], "entry"
for line in s[i:j].splitlines():
    if re.match(r"^\.?LBB\w+:|^; %bb\.\d+:", line):
        blocks.append((name, cur))
        name, cur = line.split()[0], []
    elif re.match(r"^\s+[a-z_]", line) and not line.strip().startswith(";"):
        cur.append(line.split()[0])
blocks.append((name, cur))
blocks.sort(key=lambda b: -len(b[1]))
for name, ins in blocks[:top]:
    c = Counter(ins)
    print(name, len(ins))
    print("   ", ", ".join(f"{k} {v}" for k, v in c.most_common(40)))
