"""Instruction mix of every backward-branch loop of one kernel in a -save-temps .s file.
    python tools/r5/loops.py file.s KERNEL_SUBSTRING"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
names = [m.group(1) for m in re.finditer(r"^(_Z\w+):", s, re.M) if sys.argv[2] in m.group(1)]
name = names[0]
st = s.find(name + ":")
body = s[st:s.find(".Lfunc_end", st)].split("\n")
labels = {}
for i, l in enumerate(body):
    m = re.match(r"^(\.LBB\w+):", l)
    if m:
        labels[m.group(1)] = i


def kind(x):
    for p in ("v_mfma", "ds_read", "ds_add", "ds_write", "scratch_", "global_", "s_waitcnt", "s_nop"):
        if x.startswith(p):
            return p
    return "valu" if x.startswith("v_") else "salu" if x.startswith("s_") else x


print(name[:90])
for i, l in enumerate(body):
    m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", l)
    if not m:
        continue
    t = m.group(1) or m.group(2)
    if t in labels and labels[t] < i and i - labels[t] > 40:
        seg = body[labels[t]:i + 1]
        ins = [x.strip().split()[0] for x in seg if x.strip() and not x.strip().startswith((".", ";")) and not x.strip().endswith(":")]
        c = Counter(kind(x) for x in ins)
        print(f"  loop {t} lines {labels[t]}-{i}: {len(ins)} insns {dict(c.most_common(12))}")
