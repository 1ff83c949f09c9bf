#!/usr/bin/env python3
"""Static check of the fused loop's untracked action-row loads (fs_kernels.hip, row_load).

The fused kernels load the action rows of later ticks with inline-asm `global_load_ubyte`s that
the compiler does not track, and make each row resident with an inline-asm `s_waitcnt vmcnt(N)`
followed by a `v_mov_b32` that copies the row out of the load's register.  That is only correct
if, on every path through the code, the load's destination register is neither read nor
overwritten between the load and that wait.  This tool checks exactly that on the gfx950
assembly (hipcc --cuda-device-only -S), for every kernel that contains such loads:

  python tools/check_async_loads.py [path/to/fs_kernels.hip [extra hipcc flags ...]]

It builds each kernel's control-flow graph from the labels and branches, and propagates the set
of registers with a load in flight (a may-analysis: union at joins) to a fixed point.  A register
leaves the set at the wait's `v_mov_b32 X, R` (inside the asm block that starts with the
`s_waitcnt`) or at a kernel-final `s_waitcnt vmcnt(0)` asm block.  Any other instruction that
reads or writes a register in the set is reported.

The same propagation also proves the wait counts.  `s_waitcnt vmcnt(N)` returns once at most N
vector memory operations are outstanding, and gfx9 retires them in issue order, so a load is
resident at such a wait only if at least N vector memory instructions (global_ / buffer_ /
flat_ / scratch_ loads, stores and atomics, LDS-DMA included) were issued after it.  Each
register in flight carries the MINIMUM count of those over every path that reaches a point
(min at joins, capped), and a wait whose immediate exceeds the count of a register it copies
out is reported.  Exit status 1 on any finding.
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

REG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")
ALL_READ = ("global_store", "buffer_store", "flat_store", "ds_write", "ds_add", "ds_or", "ds_and", "s_",
            "global_atomic", "buffer_atomic")
DST_ALSO_READ = ("v_mac_", "v_fmac_", "v_dot", "v_mfma", "v_movreld")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def parse_instr(line):
    """(mnemonic, written VGPRs, read VGPRs) of one instruction line."""
    code = line.split(";")[0].strip()
    if not code or code.endswith(":") or code.startswith("."):
        return None
    parts = code.split(None, 1)
    mn = parts[0]
    ops = parts[1] if len(parts) > 1 else ""
    opl = [o.strip() for o in re.split(r",(?![^\[]*\])", ops)] if ops else []
    if mn.startswith(ALL_READ) or mn.startswith("v_cmp") or mn.startswith("v_readlane") or \
            mn.startswith("v_readfirstlane"):
        return mn, set(), regs(ops)
    if not opl:
        return mn, set(), set()
    dst = regs(opl[0])
    src = regs(",".join(opl[1:]))
    m = re.search(r"op_sel_hi:\[([01,]+)\]", ops)
    if mn.startswith("v_pk_") and m and "op_sel:" not in ops:
        # a packed source whose op_sel_hi bit is 0 feeds its low register to both halves: the high
        # register of that pair is not read
        hi = [int(x) for x in m.group(1).split(",")]
        src = set()
        for i, o in enumerate(opl[1:1 + len(hi)]):
            r = regs(o)
            if hi[i] == 0 and len(r) == 2:
                r = {min(r)}
            src |= r
        for o in opl[1 + len(hi):]:
            src |= regs(o)
    if mn.startswith(DST_ALSO_READ) or ("_dpp" in mn and "bound_ctrl:1" not in ops):
        src |= dst
    return mn, dst, src


def kernels(asm):
    """{name: [lines]} for every kernel function in the assembly: from its label to its
    .Lfunc_end label (a kernel can hold several s_endpgm, e.g. an early exit of idle lanes)."""
    out, cur, name = {}, None, None
    for line in asm.splitlines():
        m = re.match(r"^(_Z\S+):\s*;", line)
        if m:
            name, cur = m.group(1), []
            out[name] = cur
            continue
        if cur is not None:
            if line.startswith(".Lfunc_end"):
                cur = None
                continue
            cur.append(line)
    return out


def blocks(lines):
    """Basic blocks: list of (label, [items], [successor labels]); items are instruction lines
    and ('asm', [lines]) groups for inline-asm blocks."""
    items, label = [], "entry"
    bbs = []
    cur = []
    in_asm = None
    for line in lines:
        s = line.strip()
        if s.startswith(";;#ASMSTART"):
            in_asm = []
            continue
        if s.startswith(";;#ASMEND"):
            cur.append(("asm", in_asm))
            in_asm = None
            continue
        if in_asm is not None:
            if s and not s.startswith(";"):
                in_asm.append(s)
            continue
        m = re.match(r"^(\.LBB\d+_\d+|%bb\.\d+):", s) or re.match(r"^; (%bb\.\d+):", s)
        if m:
            bbs.append([label, cur])
            label, cur = m.group(1), []
            continue
        if s and not s.startswith(";") and not s.startswith("."):
            cur.append(s)
    bbs.append([label, cur])
    # successors
    out = []
    for i, (lab, its) in enumerate(bbs):
        succ = []
        fall = True
        for it in its:
            if isinstance(it, tuple):
                continue
            mn = it.split()[0]
            if mn.startswith("s_cbranch"):
                succ.append(it.split()[1])
            elif mn == "s_branch":
                succ.append(it.split()[1])
                fall = False
            elif mn == "s_endpgm":
                fall = False
        if fall and i + 1 < len(bbs):
            succ.append(bbs[i + 1][0])
        out.append((lab, its, succ))
    return out


VMEM = ("global_", "buffer_", "flat_", "scratch_")
CAP = 1 << 10  # counts saturate here (enough for any wait immediate; keeps loops finite)


def is_vmem(mnemonic):
    return mnemonic.startswith(VMEM)


def prune_if_else(bbs):
    """The two exec-mask skips of one divergent if / else cannot both be taken: the then-part's
    skip means its mask (exec & cond) was empty, and the else-part then runs with the whole
    incoming mask, which is not empty (a wave that reaches code has live lanes).  The compiler's
    forms are

        B:  s_and_saveexec_b64 sX, cond ; s_xor_b64 sY, exec, sX ; ... s_cbranch_execz E
            (or s_cbranch_execnz T, the then-part elsewhere, falling through to E when empty)
        E:  s_andn2_saveexec_b64 sZ, sY ; s_cbranch_execz J      (or s_cbranch_execnz X, else-part
            (or s_or_saveexec_b64 sZ, sY ; s_xor_b64 exec, exec, sZ ; s_cbranch_execz J)   elsewhere)

    so B's then-empty edge is redirected to a copy of E without its else-empty edge.  (Without
    this, the wait counts would be checked on a path where neither half of env_step's if / else
    stores.)"""
    index = {lab: i for i, (lab, _, _) in enumerate(bbs)}
    extra = []
    for i, (lab, its, succ) in enumerate(bbs):
        code = [x for x in its if isinstance(x, str)]
        if not code or not code[-1].startswith(("s_cbranch_execz", "s_cbranch_execnz")):
            continue
        xor = [x for x in code if x.startswith("s_xor_b64") and ", exec, " in x]
        if not xor:
            continue
        if code[-1].startswith("s_cbranch_execz"):
            e_lab = code[-1].split()[1]  # the taken edge: the then-part was empty
        else:
            e_lab = bbs[i + 1][0] if i + 1 < len(bbs) else None  # the fall-through edge
        if e_lab not in index:
            continue
        mask = xor[-1].split()[1].rstrip(",")
        _, e_its, e_succ = bbs[index[e_lab]]
        e_code = [x for x in e_its if isinstance(x, str)]
        # the else header: s_andn2_saveexec_b64 sZ, sY (exec = sY & ~exec), or s_or_saveexec_b64
        # sZ, sY; s_xor_b64 exec, exec, sZ (exec = sY when the then-part was skipped)
        if len(e_code) < 2 or not e_code[0].startswith(("s_andn2_saveexec_b64", "s_or_saveexec_b64")) or \
                e_code[0].split(",")[-1].strip() != mask:
            continue
        need_xor = e_code[0].startswith("s_or_saveexec_b64")
        saved = e_code[0].split()[1].rstrip(",")
        empty_to = None
        for x in e_code[1:]:  # instructions that leave exec alone may sit in between
            if x.startswith(("s_cbranch_execz", "s_cbranch_execnz")):
                if not need_xor:
                    if x.startswith("s_cbranch_execz"):
                        empty_to = x.split()[1]
                    else:  # taken when the else mask is live: empty falls through
                        k = index[e_lab]
                        empty_to = bbs[k + 1][0] if k + 1 < len(bbs) else None
                break
            if x.replace(" ", "") == "s_xor_b64exec,exec," + saved and need_xor:
                need_xor = False
                continue
            if "exec" in x or x.startswith(("s_cbranch", "s_branch", "s_endpgm")):
                break
        if empty_to is None:
            continue
        copy = e_lab + "#then-skipped"
        if copy not in index and all(c[0] != copy for c in extra):
            extra.append((copy, e_its, [x for x in e_succ if x != empty_to] or e_succ))
        bbs[i] = (lab, its, [copy if x == e_lab else x for x in succ])
    return bbs + extra


def check_kernel(name, lines):
    bbs = prune_if_else(blocks(lines))
    index = {lab: i for i, (lab, _, _) in enumerate(bbs)}
    if not any(isinstance(it, tuple) and any(x.startswith("global_load") for x in it[1]) for _, its, _ in bbs
               for it in its):
        return None
    # per block entry: {register in flight: min VMEM instructions issued after its load, any path}
    state_in = {lab: {} for lab, _, _ in bbs}
    findings = set()
    work = [bbs[0][0]]
    seen_once = set()

    def issued(pend):
        for r in pend:
            pend[r] = min(CAP, pend[r] + 1)

    while work:
        lab = work.pop()
        _, its, succ = bbs[index[lab]]
        pend = dict(state_in[lab])
        for it in its:
            if isinstance(it, tuple):
                body = it[1]
                if body and body[0].startswith("global_load"):
                    issued(pend)
                    for r in regs(body[0].split(",")[0]):
                        pend[r] = 0
                elif body and body[0].startswith("s_waitcnt vmcnt"):
                    m = re.match(r"s_waitcnt vmcnt\((\d+)\)", body[0])
                    need = int(m.group(1)) if m else 0
                    if need == 0 and len(body) == 1:
                        pend.clear()  # the kernel-final wait
                    for x in body[1:]:
                        p = parse_instr(x)
                        if p and p[0] == "v_mov_b32":
                            for r in p[2] & set(pend):
                                if pend[r] < need:
                                    findings.add("%s [%s]: vmcnt(%d) copies v%d after only %d vector memory "
                                                 "instructions on some path: %s" % (name, lab, need, r, pend[r], x))
                                del pend[r]
                            if p[1] & set(pend):
                                findings.add("%s: asm copy writes a register in flight: %s" % (name, x))
                else:
                    for x in body:
                        p = parse_instr(x)
                        if p and (p[1] | p[2]) & set(pend):
                            findings.add("%s: asm touches a register in flight: %s" % (name, x))
                        if p and is_vmem(p[0]):
                            issued(pend)
                continue
            p = parse_instr(it)
            if not p:
                continue
            hit = (p[1] | p[2]) & set(pend)
            if hit:
                findings.add("%s [%s]: %s touches in-flight v%s" % (name, lab, it, sorted(hit)))
            if is_vmem(p[0]):
                issued(pend)
        for s_ in succ:
            if s_ not in state_in:
                continue
            old = state_in[s_]
            new = dict(old)
            for r, c in pend.items():
                new[r] = min(c, new[r]) if r in new else c
            if new != old or s_ not in seen_once:
                state_in[s_] = new
                seen_once.add(s_)
                work.append(s_)
    return findings


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "footsies_gym_amd", "csrc", "fs_kernels.hip")
    extra = sys.argv[2:]
    sys.path.insert(0, ROOT)
    from footsies_gym_amd import build as B
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        subprocess.run([B._hipcc(), "--offload-arch=" + B.ARCH, *B.flags_for(src), *extra, "-I", os.path.join(ROOT, "include"),
                        "-I", B.CSRC, "--cuda-device-only", "-S", "-o", out, src], check=True,
                       stderr=subprocess.DEVNULL)
        asm = open(out).read()
    checked, bad = 0, []
    for name, lines in kernels(asm).items():
        f = check_kernel(name, lines)
        if f is None:
            continue
        checked += 1
        bad += sorted(f)
    for b in bad:
        print(b)
    print("%d kernels with untracked row loads checked, %d findings" % (checked, len(bad)))
    sys.exit(1 if bad or not checked else 0)


if __name__ == "__main__":
    main()
