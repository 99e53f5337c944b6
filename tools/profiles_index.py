"""Regenerate profiles/README.md's file index (the header paragraph is kept)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(ROOT, "profiles")
readme = os.path.join(P, "README.md")
head = open(readme).read().split("\n## ")[0].rstrip() + "\n"
groups = {}
for f in sorted(os.listdir(P)):
    if f == "README.md":
        continue
    m = re.match(r"(r\d\d)", f)
    groups.setdefault(m.group(1) if m else "other", []).append(f)
out = [head]
for k in sorted(groups, key=lambda k: (k != "other", k)):
    out.append(f"\n## {k}\n")
    out.extend(f"- `{f}`" for f in groups[k])
open(readme, "w").write("\n".join(out) + "\n")
print(sum(len(v) for v in groups.values()), "files")
