"""Instruction mix of one kernel in a hipcc -S listing, overall and for the hottest loop.

usage: python tools/asm_mix.py listing.s <mangled-kernel-name>
"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
name = sys.argv[2]
i = s.index("\n" + name + ":") + 1
j = s.index(".Lfunc_end", i)
lines = s[i:j].split("\n")


def cls(op):
    if re.match(r"v_(fma|fmac|add|mul|div|rcp|max|min|cndmask)_f64|v_(fma|add|mul)_f64", op) or op.endswith("_f64"):
        return "valu_f64"
    if op.startswith("v_"):
        return "valu_other"
    if op.startswith("s_"):
        return "salu/branch"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    return "other"


blocks = collections.OrderedDict()
cur = "entry"
blocks[cur] = []
order = [cur]
for ln in lines:
    m = re.match(r"^(\.LBB\S+):", ln)
    if m:
        cur = m.group(1)
        blocks[cur] = []
        order.append(cur)
        continue
    t = ln.strip()
    if not t or t.startswith((";", ".")):
        continue
    blocks[cur].append(t.split()[0])
tot = collections.Counter(op for b in blocks.values() for op in b)
mix = collections.Counter()
for op, n in tot.items():
    mix[cls(op)] += n
print("static instructions:", sum(tot.values()), dict(mix))
print("top VALU ops:", [(o, n) for o, n in tot.most_common() if o.startswith("v_")][:30])
