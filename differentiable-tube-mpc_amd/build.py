"""Build libdtmpc.so (HIP, gfx950) in-tree: differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt/libdtmpc.so.

Plain hipcc, no build system: the translation units compiled in parallel, then linked --
csrc/dtmpc_kernels.hip (paper path + per-function entry points), csrc/dtmpc_fast.hip (the fused tube step of
the paper configuration), csrc/dtmpc_fast_ilqr.hip (its solver as the standalone batched iLQR), csrc/dtmpc_fast_general.hip (the
general path's solves on it), csrc/dtmpc_general.hip (general IFT
path), csrc/dtmpc_receding.hip (receding-horizon nominal MPC driver), csrc/dtmpc_control.hip (tanh-box
control map + cost derivatives), csrc/dtmpc_ocp.hip (tape cost of core/ocp.py), csrc/dtmpc_systems.hip
(per-point kernels of the reference's per-function API: dynamics, h, barriers, Jacobians, clamp, cost
derivatives).
"""
from __future__ import annotations

import hashlib
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRCS = [os.path.join(HERE, "csrc", f)
        for f in ("dtmpc_kernels.hip", "dtmpc_fast.hip", "dtmpc_fast_ilp.hip", "dtmpc_fast64.hip", "dtmpc_fast64_ilp.hip",
                  "dtmpc_fast64_ilqr.hip", "dtmpc_fast64_general.hip", "dtmpc_fast_ilqr.hip", "dtmpc_fast_general.hip", "dtmpc_general.hip", "dtmpc_receding.hip",
                  "dtmpc_control.hip", "dtmpc_ocp.hip", "dtmpc_systems.hip")]
DEPS = [os.path.join(HERE, "csrc", f) for f in ("dtmpc_device.hpp", "dtmpc_solver.hpp", "dtmpc_general.hpp",
                                                 "dtmpc_host.hpp", "dtmpc_ls_pk.hpp")] + [
    os.path.join(os.path.dirname(HERE), "include", h) for h in ("dtmpc.h", "dtmpc_control.h", "dtmpc_systems.h")
]
OUT = os.path.join(HERE, "diff_tube_mpc_strict_pt", "libdtmpc.so")
CACHE = os.path.join(HERE, "build", "obj")  # object cache keyed by the command line + source texts
ARCH = os.environ.get("DTMPC_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", f"--offload-arch={ARCH}", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function"]
# per-unit flags: the one-lane tube kernels (one wave per SIMD at the headline batch, nothing to hide a stall behind) and
# the f32 two-lane ones with LLVM's iterative ILP scheduler -- same-box A/B in profiles/r06/ab_sched.txt; the four-lane
# forms lost with it
# and the f32 standalone-iLQR / receding unit (config 2 -1.3 %, receding -0.8 %; its f64 twin lost 1.2 % and keeps the
# default) and the f32 general-path unit (general IFT step -1.1 %)
UNIT_FLAGS = {u: ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]
              for u in ("dtmpc_fast_ilp", "dtmpc_fast64_ilp", "dtmpc_fast_ilqr", "dtmpc_fast_general")}


def _lib_key() -> str:
    """Content key of the product library: every unit's command line and source texts (not mtimes: a
    source edited while a build runs must not leave a stale library that looks up to date)."""
    h = hashlib.sha256(open(__file__, "rb").read())
    for src in SRCS:
        tu = os.path.splitext(os.path.basename(src))[0]
        h.update(_key([HIPCC, *FLAGS, *UNIT_FLAGS.get(tu, []), "-c"], src).encode())
    return h.hexdigest()


def up_to_date() -> bool:
    if not os.path.exists(OUT) or not os.path.exists(OUT + ".key"):
        return False
    return open(OUT + ".key").read().strip() == _lib_key()


FAST = os.path.join(HERE, "csrc", "dtmpc_fast.hip")  # included by dtmpc_fast_ilqr.hip / dtmpc_fast_general.hip


def _key(cmd, src) -> str:
    h = hashlib.sha256(" ".join(cmd).encode())
    for p in [src, *DEPS, *([FAST] if os.path.basename(src).startswith("dtmpc_fast") else [])]:
        h.update(open(p, "rb").read())
    return h.hexdigest()[:24]


PRODUCT_OBJS = os.path.join(CACHE, "product_objs.txt")  # the product library's objects, one per line


def build(force: bool = False, variant: str = "", defines=(), only=(), on_product: bool = False) -> str:
    """Build the library.  ``variant`` (with extra ``-D`` defines) writes libdtmpc_<variant>.so next to
    the product library, for A/B kernel experiments loaded through DTMPC_LIBRARY; it never replaces
    libdtmpc.so.  ``only`` restricts the defines / extra flags to the named translation units (e.g.
    ``dtmpc_fast``); objects are cached under build/obj by command line and source text, so a variant
    recompiles only the units its flags reach.  ``on_product`` (variants with ``only``): the units not named
    are taken from the last product build as they are (build/obj/product_objs.txt), never recompiled -- an A/B
    of one unit against exactly the product library's other objects."""
    out = OUT if not variant else OUT.replace("libdtmpc.so", f"libdtmpc_{variant}.so")
    if not variant and not force and up_to_date():
        return out
    key = _lib_key() if not variant else None  # the sources as they are when the units start compiling
    os.makedirs(CACHE, exist_ok=True)
    objs = []
    procs = []
    prod = {}
    if on_product:
        if not variant or not only:
            raise ValueError("on_product needs a variant and the units it rebuilds (only)")
        for o in open(PRODUCT_OBJS).read().split():
            prod[os.path.basename(o).split(".")[0]] = o
    for src in SRCS:
        tu = os.path.splitext(os.path.basename(src))[0]
        reach = not only or tu in only
        if on_product and not reach:
            objs.append(prod[tu])
            continue
        extra = os.environ.get("DTMPC_EXTRA_FLAGS", "").split() if variant and reach else []
        defs = [f"-D{d}" for d in defines] if reach else []
        # DTMPC_NO_UNIT_FLAGS=1 (variants only): the units without their UNIT_FLAGS, for the A/B that keeps them
        uf = [] if variant and os.environ.get("DTMPC_NO_UNIT_FLAGS") == "1" and reach else UNIT_FLAGS.get(tu, [])
        cmd = [HIPCC, *FLAGS, *uf, *extra, *defs, "-c"]
        obj = os.path.join(CACHE, f"{tu}.{_key(cmd, src)}.o")
        objs.append(obj)
        if os.path.exists(obj):  # content-keyed: safe to reuse even under --force
            continue
        full = [*cmd, "-o", obj + ".tmp", src]
        print("[build]", " ".join(full), flush=True)
        procs.append((subprocess.Popen(full), obj, cmd, src))
    if any([p.wait() != 0 for p, *_ in procs]):
        raise subprocess.CalledProcessError(1, "hipcc")
    for _, obj, cmd, src in procs:
        # hipcc reads the source once for the device pass and again for the host pass, minutes apart: an object whose
        # sources changed meanwhile would pair one text's kernels with another's launchers under the first text's key
        if os.path.basename(obj).split(".")[1] != _key(cmd, src):
            os.remove(obj + ".tmp")
            raise RuntimeError(f"{src} or a header it includes changed during the build; run it again")
        os.replace(obj + ".tmp", obj)
    if not variant:  # the product: no f64 fused kernel may keep anything in scratch (check_resources)
        import json

        rep = check_resources(objs, strict=False)
        with open(os.path.join(CACHE, "resources.json"), "w") as f:
            json.dump(rep, f, indent=1, sort_keys=True)
        bad = [(k, v["scratch"]) for r in rep.values() for k, v in r.items() if v.get("scratch", 0)]
        if bad and os.environ.get("DTMPC_RESOURCE_STRICT", "1") != "0":
            raise RuntimeError("f64 fused kernels with a private segment (scratch): " +
                               ", ".join(f"{k} ({b} B)" for k, b in bad))
        # and no 128-bit record store of a fused kernel may have its data registers written inside its two wait
        # states (the store-data hazard, csrc/dtmpc_fast.hip st128; profiles/r05/store_hazard.txt)
        haz, vh, fc = {}, {}, {}
        for o in objs:
            tu = os.path.basename(o).split(".")[0]
            if tu.startswith("dtmpc_fast"):
                haz[tu] = [list(h) for h in store_hazards(o)]
                vh[tu] = [list(h) for h in valu_hazards(o)]
            fc[tu] = [list(h) for h in flow_copies(o)]  # every unit: the generic kernels branch per lane as well
        with open(os.path.join(CACHE, "flow_copies.json"), "w") as f:
            json.dump(fc, f, indent=1, sort_keys=True)
        nf = sum(len(v) for v in fc.values())
        if nf and os.environ.get("DTMPC_RESOURCE_STRICT", "1") != "0":
            raise RuntimeError(f"{nf} vector-register writes in divergent flow blocks (build/obj/flow_copies.json): "
                               + ", ".join(sorted({h[0] for v in fc.values() for h in v}))[:2000])
        with open(os.path.join(CACHE, "store_hazards.json"), "w") as f:
            json.dump(haz, f, indent=1, sort_keys=True)
        with open(os.path.join(CACHE, "valu_hazards.json"), "w") as f:
            json.dump(vh, f, indent=1, sort_keys=True)
        nh = sum(len(v) for v in haz.values())
        if nh and os.environ.get("DTMPC_RESOURCE_STRICT", "1") != "0":
            raise RuntimeError(f"{nh} 128-bit stores with their data registers overwritten inside the hazard window "
                               "(build/obj/store_hazards.json)")
        nv = sum(len(v) for v in vh.values())
        if nv and os.environ.get("DTMPC_RESOURCE_STRICT", "1") != "0":
            raise RuntimeError(f"{nv} wait-state hazards (DPP / readlane / SGPR->VMEM / trans) in the fused kernels "
                               "(build/obj/valu_hazards.json)")
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out + ".tmp", *objs]
    print("[build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    if key is not None:
        with open(out + ".key", "w") as f:
            f.write(key)
        with open(PRODUCT_OBJS, "w") as f:
            f.write("\n".join(objs) + "\n")
    return out


LLVM = "/opt/rocm/lib/llvm/bin"
# f64 fused units: every kernel must run without a private segment (round 5) -- the f64
# defects of rounds 3-4 (wrong results, run-to-run differences, an illegal address) came only from f64 fused
# kernels whose per-lane divergent loops spilled VGPRs to scratch or kept results in scratch through a pointer
RESOURCE_CHECKED = ("dtmpc_fast64", "dtmpc_fast64_ilp", "dtmpc_fast64_ilqr", "dtmpc_fast64_general")


def kernel_resources(obj: str) -> dict:
    """{kernel: {"scratch": private_segment_fixed_size, "sgpr_spill": .., "vgpr_spill": ..}} of the gfx950 code
    object inside a hipcc object file (its .hip_fatbin section, unbundled; the code-object metadata notes)."""
    import re
    import tempfile

    with tempfile.TemporaryDirectory() as d:
        co = _code_object(obj, d)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                               text=True).stdout
    out, cur = {}, None
    for line in notes.splitlines():
        m = re.match(r"\s+\.name:\s+(\S+)", line)
        if m:
            cur = out.setdefault(m.group(1), {})
            continue
        for key, field in (("scratch", "private_segment_fixed_size"), ("sgpr_spill", "sgpr_spill_count"),
                           ("vgpr_spill", "vgpr_spill_count")):
            m = re.match(r"\s+\.%s:\s+(\d+)" % field, line)
            if m and cur is not None:
                cur[key] = int(m.group(1))
    return out


def _code_object(obj: str, d: str) -> str:
    fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "dev.co")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(d, "x.o")],
                   check=True, capture_output=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    f"--targets=hipv4-amdgcn-amd-amdhsa--{ARCH}", f"--output={co}"], check=True, capture_output=True)
    return co


def _vregs(tok: str):
    """The VGPR numbers of an operand token (v7, v[6:9])."""
    import re

    m = re.fullmatch(r"v(\d+)", tok) or re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if not m:
        return set()
    lo = int(m.group(1))
    hi = int(m.group(2)) if m.lastindex == 2 else lo
    return set(range(lo, hi + 1))


def store_hazards(obj: str) -> list:
    """128-bit (and 96-bit) buffer stores whose data VGPRs a VALU instruction writes within the two wait states
    after the store (the gfx950 store-data hazard the compiler does not pad for buffer stores with an SGPR soffset,
    csrc/dtmpc_fast.hip st128): [(kernel, store line, offending line)] of the code object in a hipcc object."""
    import tempfile

    with tempfile.TemporaryDirectory() as d:
        co = _code_object(obj, d)
        dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", f"--mcpu={ARCH}", "--no-show-raw-insn",
                              "--no-leading-addr", co], check=True, capture_output=True, text=True).stdout
    return scan_store_hazards(dis)


def scan_store_hazards(dis: str) -> list:
    """store_hazards on a disassembly text (llvm-objdump -d): [(kernel, store line, offending line)]."""
    import re

    out, kern = [], None
    lines = dis.splitlines()
    for i, line in enumerate(lines):
        m = re.match(r"^(\S+):$", line.strip()) if line and not line.startswith((" ", "\t")) else None
        if m or re.match(r"^[0-9a-f]+ <(\S+)>:", line):
            kern = (m.group(1) if m else re.match(r"^[0-9a-f]+ <(\S+)>:", line).group(1))
            continue
        t = line.split()
        if not t or not re.match(r"buffer_store_dwordx[34]$", t[0]):
            continue
        data = _vregs(t[1].rstrip(","))
        waits = 0
        for nxt in lines[i + 1:i + 6]:
            u = nxt.split()
            if not u or u[0].endswith(":"):
                break
            if u[0] == "s_nop":
                waits += int(u[1], 0) + 1
            elif u[0].startswith("v_"):
                if _vregs(u[1].rstrip(",")) & data:
                    out.append((kern, line.strip(), nxt.strip()))
                    break
                waits += 1
            else:
                waits += 1
            if waits >= 2:
                break
    return out


# gfx9 / CDNA4 wait-state rules the compiler pads for its own instructions but not around inline assembly (an asm
# statement is one opaque instruction to hipcc: cdna_hip_programming.md section 5.7 item 2) -- checked on the final
# code of every fused kernel, whatever produced it (widen the scan beyond the store-data hazard).
# (class, wait states the consumer needs after the producer)
VALU_HAZARDS = {
    "VALU->DPP": 2,            # a VALU write of a VGPR, then a DPP instruction reading it
    "VALU->READLANE": 1,       # a VALU write of a VGPR, then v_readlane / v_readfirstlane reading it
    "VALU_SGPR->VMEM": 5,      # a VALU write of an SGPR (v_readlane, v_readfirstlane, v_cmp, carry-out), then a
                               # buffer / global instruction reading it (descriptor, soffset, saddr)
    "VALU_SGPR->LANESEL": 4,   # the same SGPR as the lane select of v_readlane / v_writelane
    "TRANS->VALU": 1,          # a transcendental (v_exp / log / rcp / rsq / sqrt / sin / cos), then a non-trans VALU reading its result
}
_TRANS = r"^v_(exp|log|rcp|rsq|sqrt|sin|cos)_(f16|f32|f64|legacy|iflag)"


def _sregs(tok: str):
    """The SGPR numbers of an operand token (s7, s[6:9]); vcc is s[106:107]."""
    import re

    tok = tok.strip().rstrip(",")
    if tok in ("vcc", "vcc_lo"):
        return {106, 107} if tok == "vcc" else {106}
    m = re.fullmatch(r"s(\d+)", tok) or re.fullmatch(r"s\[(\d+):(\d+)\]", tok)
    if not m:
        return set()
    lo = int(m.group(1))
    hi = int(m.group(2)) if m.lastindex == 2 else lo
    return set(range(lo, hi + 1))


def _operands(ins: str):
    """(opcode, operand tokens) of one disassembled instruction (modifiers such as quad_perm: / offen dropped)."""
    import re

    ins = ins.split("//")[0].strip()
    parts = ins.split(None, 1)
    if len(parts) < 2:
        return parts[0] if parts else "", []
    body = re.split(r"\s(?:quad_perm|row_\w+|wave_\w+|offen|idxen|offset|bank_mask|bound_ctrl|sc0|sc1|nt|lds|glc|slc)",
                    " " + parts[1])[0]
    return parts[0], [t for t in re.split(r",\s*", body.strip()) if t]


def scan_valu_hazards(dis: str, window: int = 6) -> list:
    """VALU_HAZARDS on a disassembly text (llvm-objdump -d): [(class, kernel, producer, consumer, wait states seen)].
    Straight-line windows in program order (a branch counts as one wait state and the scan continues on the
    fall-through path, which over-approximates: a hit is a site to read, and the product has none)."""
    import re

    out, kern, prog = [], None, []
    for line in dis.splitlines():
        m = re.match(r"^<(\S+)>:", line.strip()) if line and not line.startswith((" ", "\t")) else None
        m = m or re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            kern = m.group(1)
            continue
        if line.startswith("\t") and kern:
            prog.append((kern, line.strip()))
    n = len(prog)
    for i, (k, ins) in enumerate(prog):
        op, ops = _operands(ins)
        if not op.startswith("v_") or not ops:
            continue
        dv, ds = set(), set()
        if op.startswith(("v_readlane", "v_readfirstlane", "v_cmp")):
            ds = _sregs(ops[0])
        else:
            dv = _vregs(ops[0])
            if len(ops) > 1 and re.match(r"v_(add|sub|addc|subb|subrev)_co|v_div_scale|v_mad_[iu]64", op):
                ds = _sregs(ops[1])
        trans = re.match(_TRANS, op) is not None
        w = 0
        for j in range(i + 1, min(n, i + 1 + window)):
            k2, ins2 = prog[j]
            if k2 != k:
                break
            op2, ops2 = _operands(ins2)
            if op2 == "s_endpgm":
                break
            rv, rs = set(), set()
            for t in ops2[1:]:
                rv |= _vregs(t.rstrip(","))
                rs |= _sregs(t)
            if op2.startswith(("buffer_store", "global_store")) and ops2:
                rv |= _vregs(ops2[0].rstrip(","))
            hit = None
            if op2.startswith(("buffer_", "global_")):
                srs = set()
                for t in ops2:
                    srs |= _sregs(t)
                if ds & srs and w < VALU_HAZARDS["VALU_SGPR->VMEM"]:
                    hit = "VALU_SGPR->VMEM"
            elif ("_dpp" in op2 or "quad_perm" in ins2 or "row_" in ins2) and dv & rv and w < VALU_HAZARDS["VALU->DPP"]:
                hit = "VALU->DPP"
            elif op2.startswith(("v_readlane", "v_readfirstlane")) and len(ops2) > 1:
                if dv & _vregs(ops2[1].rstrip(",")) and w < VALU_HAZARDS["VALU->READLANE"]:
                    hit = "VALU->READLANE"
                elif len(ops2) > 2 and ds & _sregs(ops2[2]) and w < VALU_HAZARDS["VALU_SGPR->LANESEL"]:
                    hit = "VALU_SGPR->LANESEL"
            elif op2.startswith("v_writelane") and len(ops2) > 2 and ds & _sregs(ops2[2]) and \
                    w < VALU_HAZARDS["VALU_SGPR->LANESEL"]:
                hit = "VALU_SGPR->LANESEL"
            elif trans and op2.startswith("v_") and not re.match(_TRANS, op2) and dv & rv and w < VALU_HAZARDS["TRANS->VALU"]:
                hit = "TRANS->VALU"
            if hit:
                out.append((hit, k, ins.split("//")[0].strip(), ins2.split("//")[0].strip(), w))
            w += int(ops2[0], 0) + 1 if op2 == "s_nop" and ops2 else 1
            if w >= 5:
                break
    return out


def valu_hazards(obj: str) -> list:
    """scan_valu_hazards on the gfx950 code object inside a hipcc object file."""
    import tempfile

    with tempfile.TemporaryDirectory() as d:
        co = _code_object(obj, d)
        dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", f"--mcpu={ARCH}", "--no-show-raw-insn",
                              "--no-leading-addr", co], check=True, capture_output=True, text=True).stdout
    return scan_valu_hazards(dis)


def _listing(dis: str):
    """{kernel: [(instruction, byte offset, branch-target offset or None)]} of an llvm-objdump -d text."""
    import re

    out, cur = {}, None
    for line in dis.splitlines():
        m = re.match(r"^<(\S+)>:", line.strip()) if line and not line.startswith((" ", "\t")) else None
        m = m or re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            cur = out.setdefault(m.group(1), [])
            continue
        if cur is None or not line.startswith("\t"):
            continue
        a = re.search(r"// ([0-9A-F]+):", line)
        if not a:
            continue
        t = re.search(r"<\S+\+0x([0-9a-f]+)>", line)
        cur.append((line.split("//")[0].strip(), int(a.group(1), 16), int(t.group(1), 16) if t else None))
    for k, ins in out.items():
        if ins:
            b = ins[0][1]
            out[k] = [(x, a - b, (t - 0) if t is not None else None) for x, a, t in ins]
    return out


def scan_flow_copies(dis: str) -> list:
    """Vector-register writes in the FLOW block of a divergent if / else (round 6, profiles/r06/flow_copy_root_cause.txt):
    after `s_and_saveexec_b64 sX, vcc ; s_xor_b64 sX, exec, sX ; s_cbranch_execz FLOW`, the block FLOW is entered on
    both control paths but runs with the THEN lanes' exec mask until its `s_andn2_saveexec_b64` switches to the else
    lanes -- so a copy the register allocator places there (a live-range split of a value defined before the branch)
    reaches the then-lanes only, and the else-lanes later read the register's stale content.  v_writelane /
    v_readlane (exec-independent SGPR spills) are not writes of this kind.  [(kernel, if offset, instruction)]."""
    out = []
    for k, ins in _listing(dis).items():
        idx = {a: i for i, (_, a, _) in enumerate(ins)}
        for i in range(len(ins) - 2):
            if not (ins[i][0].startswith("s_and_saveexec_b64") and ins[i + 1][0].startswith("s_xor_b64")
                    and "exec" in ins[i + 1][0] and ins[i + 2][0].startswith("s_cbranch_execz")):
                continue
            t = ins[i + 2][2]
            if t not in idx:
                continue
            j = idx[t]
            while j < len(ins) and not ins[j][0].startswith(("s_andn2_saveexec_b64", "s_or_saveexec_b64", "s_or_b64 exec",
                                                             "s_mov_b64 exec", "s_branch", "s_cbranch", "s_endpgm")):
                x = ins[j][0]
                if x.startswith("v_") and not x.startswith(("v_writelane", "v_readlane", "v_readfirstlane", "v_cmp")):
                    out.append((k, ins[i][1], x))
                j += 1
    return out


def flow_copies(obj: str) -> list:
    """scan_flow_copies on the gfx950 code object inside a hipcc object file."""
    import tempfile

    with tempfile.TemporaryDirectory() as d:
        co = _code_object(obj, d)
        dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", f"--mcpu={ARCH}", "--no-show-raw-insn",
                              "--no-leading-addr", co], check=True, capture_output=True, text=True).stdout
    return scan_flow_copies(dis)


def check_resources(objs, strict: bool = True) -> dict:
    """The f64 fused units' kernels and their resources; raises when one has a private segment (strict)."""
    report, bad = {}, []
    for o in objs:
        tu = os.path.basename(o).split(".")[0]
        if tu not in RESOURCE_CHECKED:
            continue
        res = kernel_resources(o)
        report[tu] = res
        bad += [(tu, k, v["scratch"]) for k, v in res.items() if v.get("scratch", 0)]
    if bad and strict:
        raise RuntimeError("f64 fused kernels with a private segment (scratch): " +
                           ", ".join(f"{k} ({s} B)" for _, k, s in bad))
    return report


if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--variant", default="")
    ap.add_argument("-D", dest="defines", action="append", default=[])
    ap.add_argument("--only", action="append", default=[], help="translation unit(s) the -D / extra flags reach")
    ap.add_argument("--on-product", action="store_true",
                    help="with --variant/--only: link the other units from the last product build as they are")
    a = ap.parse_args()
    print(build(force=a.force, variant=a.variant, defines=a.defines, only=tuple(a.only), on_product=a.on_product))
