"""Static loop census of a hipcc -S listing: for every backward branch (a loop), the instruction mix of
its body (VALU / packed VALU / transcendental / SALU / VMEM / LDS / waitcnt).  usage: isa_loops.py f.s [kernel-substr]"""
import re
import sys
from collections import Counter

src = open(sys.argv[1]).read().splitlines() if __name__ == "__main__" else []
want = sys.argv[2] if len(sys.argv) > 2 else ""
# split into functions
funcs, cur, name = {}, None, None
for ln in src:
    m = re.match(r"^([_A-Za-z0-9.$]+):\s*(;.*)?$", ln)
    if m and not m.group(1).startswith(".") and "@function" not in ln:
        if m.group(1).startswith("_Z"):
            name = m.group(1)
            cur = funcs.setdefault(name, [])
            continue
    if cur is not None:
        cur.append(ln)
TRANS = ("v_exp_f32", "v_log_f32", "v_rcp_f32", "v_sqrt_f32", "v_rsq_f32", "v_sin_f32", "v_cos_f32", "v_rcp_iflag")


def kind(op):
    if op.startswith("v_pk_"):
        return "pk"
    if op.startswith(TRANS):
        return "trans"
    if op.startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
        return "lane"
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem_st" if "store" in op else "vmem_ld"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_load") or op.startswith("s_buffer"):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    return "other"


for fn, body in (funcs.items() if __name__ == "__main__" else []):
    if want not in fn:
        continue
    lines = [l.split(";")[0].strip() for l in body]
    labels = {}
    ins = []
    for l in lines:
        m = re.match(r"^([.A-Za-z0-9_$]+):$", l)
        if m:
            labels[m.group(1)] = len(ins)
            continue
        if not l or l.startswith("."):
            continue
        ins.append(l)
    print(f"== {fn[:90]}  ({len(ins)} instructions)")
    tot = Counter(kind(i.split()[0]) for i in ins)
    print("   total:", dict(tot))
    for idx, i in enumerate(ins):
        op = i.split()[0]
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = i.split()[-1]
            if tgt in labels and labels[tgt] <= idx:
                b = ins[labels[tgt]:idx + 1]
                c = Counter(kind(x.split()[0]) for x in b)
                print(f"   loop {tgt} [{labels[tgt]}..{idx}] n={len(b)}", dict(c))
