"""Instruction mix of a kernel's innermost loop from hipcc --save-temps assembly.
    python scripts/diag/isa_mix.py <file.s> <kernel symbol substring> [loop label index]
Prints per-loop counts of instruction classes (VALU, transcendental, packed, SALU, VMEM,
SMEM, LDS, MFMA, spills, s_nop, waitcnt) for every loop (a label with a backward branch)."""
import collections
import re
import sys

path, sym = sys.argv[1], sys.argv[2]
s = open(path).read()
names = [m.group(1) for m in re.finditer(r"^(\S+):\s*(?:;.*)?$", s, re.M) if sym in m.group(1)
         and not m.group(1).startswith(".")]
name = names[0]
i = s.index(name + ":")
j = s.index(".Lfunc_end", i)
lines = [l.split(";")[0].strip() for l in s[i:j].splitlines()]
labels = {l[:-1]: n for n, l in enumerate(lines) if l.startswith(".LBB") and l.endswith(":")}


def cls(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op in ("v_exp_f32", "v_log_f32", "v_rcp_f32", "v_sqrt_f32", "v_rsq_f32"):
        return "trans"
    if op.startswith("v_pk_"):
        return "valu_pk"
    if op.startswith(("v_readlane", "v_writelane")):
        return "lane_rw(spill?)"
    if op.startswith("v_accvgpr"):
        return "accvgpr"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_nop"):
        return "s_nop"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    return "other"


for n, l in enumerate(lines):
    m = re.match(r"s_cbranch_\w+\s+(\.LBB\S+)", l)
    if m and m.group(1) in labels and labels[m.group(1)] < n:
        a = labels[m.group(1)]
        c = collections.Counter(cls(x.split()[0]) for x in lines[a + 1:n] if x and not x.startswith((".", "//")))
        print(f"loop {m.group(1)} lines {a}-{n}:", dict(sorted(c.items())))
