"""Extract one kernel's gfx950 ISA from a -save-temps .s file and summarise it.

python scripts/asm_kernel.py <file.s> <mangled-name-substring> [out.s]
Prints instruction counts by class and every scratch (spill) access with its line number.
"""
import collections
import re
import sys

src, pat = sys.argv[1], sys.argv[2]
s = open(src).read()
m = re.search(r"^(\S*" + re.escape(pat) + r"\S*):", s, re.M)
if not m:
    sys.exit("kernel not found")
a = m.start()
b = s.index(".Lfunc_end", a)
k = s[a:b]
if len(sys.argv) > 3:
    open(sys.argv[3], "w").write(k)
cls = collections.Counter()
for i, line in enumerate(k.split("\n")):
    t = line.strip()
    if not t or t.startswith(";") or t.startswith(".") or t.endswith(":"):
        continue
    op = t.split()[0]
    cls[op.split("_")[0]] += 1
    if "scratch_" in op or ("buffer_" in op and "off" in t):
        print(i, t)
print(dict(cls.most_common(12)))
