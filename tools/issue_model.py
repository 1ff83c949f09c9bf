#!/usr/bin/env python3
"""SIMD-level issue picture of the fused step kernel (measurement support).

  python tools/issue_model.py [--lib footsies_gym_amd/libfootsies.so] [--kernel MANGLED_NAME]
                              [--probe profiles/r03_valu_probe.json] [--sq profiles/r03a_sq.json]
                              [--occupancy profiles/r03_occupancy.txt] [--json profiles/r03_issue_model.json]

Two views of how much of its SIMDs the C3 kernel (two lanes per arena, 2 waves per SIMD at
65 536 arenas) uses:

* measured: the same kernel at 4 and 8 waves per SIMD (131 072 / 262 144 arenas,
  tools/occupancy_sweep.sh) reaches a plateau -- no resource but the SIMD's issue is near its
  limit there (HBM ~0.3, LDS ~0.2 busy) -- and `issue_frac` = the env-step rate at the kernel's own
  occupancy over that plateau: the share of the SIMD issue rate this instruction stream can get
  that it does get.  The rest is latency no second wave covers.
* priced: the VALU of the kernel's main loop (the backward branch spanning the most instructions:
  two ticks of the row loop) classified and priced by tools/valu_probe (SIMD cycles per
  instruction at the kernel's waves per SIMD: a plain 32-bit VOP1 / VOP2 op 2.4, VOP3-only ops
  (v_bfe, v_add3, v_bitop3, v_lshl_or ...), DPP and packed f32 4.7-5.6, a VOPC compare 5.6, a vcc
  v_cndmask right after another ~5.5).  The probe also shows the costs are not additive (one
  v_bfe_u32 among three v_add_u32 costs more than either run alone), so `valu_pipe_frac_priced`
  is an estimate; `valu_pipe_frac_if_all_fast` (every VALU at the plain-op rate) is a floor on
  the pipe time the kernel's VALU count needs.
"""
import argparse
import json
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"


def disassemble(lib):
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fatbin"), os.path.join(d, "co")
        subprocess.run([LLVM + "/llvm-objcopy", "--dump-section=.hip_fatbin=" + fat, lib], check=True)
        subprocess.run([LLVM + "/clang-offload-bundler", "--type=o", "--input=" + fat,
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co, "--unbundle"], check=True)
        return subprocess.run([LLVM + "/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True, capture_output=True,
                              text=True).stdout


INST = re.compile(r"^\s+(\S+)\s*([^/]*)//\s+([0-9A-F]+):\s+([0-9A-F ]+)")


def kernel_insts(dis, name):
    out, on = [], False
    for line in dis.splitlines():
        if line.rstrip().endswith(">:"):
            on = name in line
            continue
        m = INST.match(line) if on else None
        if m:
            out.append((int(m.group(3), 16), m.group(1), m.group(2).strip(), 4 * len(m.group(4).split())))
    return out


def main_loop(insts):
    """[start, end] indices of the standard tick loop: the backward branch spanning the most
    instructions among those whose body loads nothing 16 bytes wide from global memory.  (Since
    round 4 each fused kernel holds two tick loops, the standard one and the general-geometry
    one, which reads the boxes' y extents from kRecY.)"""
    addr = {a: i for i, (a, *_rest) in enumerate(insts)}
    loops = []
    for i, (a, mn, ops, size) in enumerate(insts):
        if mn.startswith("s_cbranch") or mn == "s_branch":
            off = int(ops.split()[0])
            off = off - 65536 if off >= 32768 else off
            tgt = a + 4 + 4 * off
            if off < 0 and tgt in addr:
                loops.append((addr[tgt], i))
    # the general-geometry loop reads kRecY (global_load_dwordx4); the standard tick has no 16-byte
    # global loads (its tables are in LDS, its row loads single bytes)
    std = [lp for lp in loops if not any(insts[j][1] == "global_load_dwordx4" for j in range(lp[0], lp[1] + 1))]
    pool = std or loops
    return max(pool, key=lambda lp: lp[1] - lp[0]) if pool else None


def reads_vcc(mn, ops):
    return mn.startswith("v_") and not mn.startswith("v_cmp") and re.search(r"\bvcc\b", ops.split(",", 1)[-1]) is not None


# plain 32-bit ops the probe runs at the fast rate in either encoding (v_add_u32 / v_add_f32 /
# v_xor / v_or runs, v_add_u32_e64 3.0, a v_mov of a literal 3.0, a v_and with a literal among adds)
FAST = re.compile(r"^v_(add|sub|subrev|xor|or|and|mov|add_f32|sub_f32|mul_f32|max|min|cndmask)_(u32|i32|b32|f32)")


def classify(mn, ops, size, prev_vcc):
    if mn.startswith("v_pk_"):
        return "pk_f32"
    if mn.startswith("v_cmp") or mn.startswith("v_cmpx"):
        return "vopc"
    if "row_" in ops or "quad_perm" in ops or "sel:" in ops:
        return "dpp_sdwa"
    if mn.startswith("v_cndmask_b32_e32") and prev_vcc:
        return "cndmask_vcc_b2b"
    if mn.startswith("v_cndmask_b32_e64") or re.search(r"(^|, )s\[?\d", ops):
        return "vop3_op"  # an SGPR-pair mask or an SGPR operand: the probe's slow kinds
    if FAST.match(mn) or mn.startswith("v_mov_b32") or mn.startswith("v_mov_b64"):
        return "fast"
    return "vop3_op"


# probe kinds (tools/valu_probe/probe.hip) that price each class; cndmask_vcc_b2b: the second of
# a pair, from "2 v_cndmask_b32 vcc + 2 v_add_u32" (4 x that rate - 3 plain ops)
PROBE_KIND = {"fast": "v_add_u32", "vop3_op": "v_bfe_u32", "dpp_sdwa": "v_mov_b32_dpp", "pk_f32": "v_pk_add_f32",
              "vopc": "v_cmp_gt_u32 vcc"}


def occupancy_plateau(path, packed=False):
    """{arenas: env-steps/s} of the two-lane kernel in an occupancy sweep log: FOOTSIES_FUSED_LANES=2
    lines of tools/ab_time.py (tools/occupancy_sweep.sh), or, for the packed-trajectory kernel, the
    `packed` rates of tools/packed_ab.py at 65 536 / 131 072 / 262 144 arenas."""
    out = {}
    if not path or not os.path.exists(path):
        return out
    pat = (r"packed\s+[\d.]+ us \(([\d.e+]+)[,)]" if packed else
           r"FUSED_LANES=2\s+C3\s+[\d.]+ us \(([\d.e+]+) env-steps/s")
    for line in open(path):
        m = re.search(pat, line)
        if m:
            out.setdefault(len(out), float(m.group(1)))
    return out


def model(lib, kernel, probe_path, sq_path, sq_kernel, occ_path):
    insts = kernel_insts(disassemble(lib), kernel)
    lo, hi = main_loop(insts)
    counts, prev_vcc = {}, False
    for a, mn, ops, size in insts[lo:hi + 1]:
        if not mn.startswith("v_") or mn.startswith(("v_readfirstlane", "v_readlane", "v_writelane")):
            continue
        c = classify(mn, ops, size, prev_vcc)
        counts[c] = counts.get(c, 0) + 1
        prev_vcc = reads_vcc(mn, ops)
    with open(probe_path) as f:
        probe = json.load(f)
    with open(sq_path) as f:
        sq = next(k for k in json.load(f)["kernels"] if k["kernel"] == sq_kernel)
    wps = sq["waves"] / 1024.0
    near = min({r["waves_per_simd"] for r in probe["runs"]}, key=lambda w: abs(w - wps))

    def rate(kind):
        return next(r["simd_cycles_per_instr"] for r in probe["runs"] if r["kind"] == kind and r["waves_per_simd"] == near)
    cost = {c: rate(k) for c, k in PROBE_KIND.items()}
    cost["cndmask_vcc_b2b"] = 4 * rate("2 v_cndmask_b32 vcc + 2 v_add_u32") - 3 * cost["fast"]
    n = sum(counts.values())
    per_valu = sum(cost[c] * counts.get(c, 0) for c in cost) / n
    pw = sq["per_wave_tick"]
    valu, quad = pw["SQ_INSTS_VALU"], pw["SQ_WAVE_CYCLES"]
    res = {
        "kernel": sq["kernel"], "envs": sq["envs"], "waves_per_simd": wps, "probe_waves_per_simd": near,
        "loop_valu_static": counts, "loop_valu_total": n,
        "simd_cycles_per_valu": {c: round(v, 3) for c, v in cost.items()},
        "mix_cycles_per_valu": round(per_valu, 3),
        "valu_per_wave_tick": round(valu, 1), "simd_cycles_per_tick": round(4.0 * quad, 1),
        "valu_pipe_frac_priced": round(wps * valu * per_valu / (4.0 * quad), 3),
        "valu_pipe_frac_if_all_fast": round(wps * valu * cost["fast"] / (4.0 * quad), 3),
        "sources": {"probe": os.path.relpath(probe_path, ROOT), "sq": os.path.relpath(sq_path, ROOT)},
    }
    occ = occupancy_plateau(occ_path, packed="packed" in kernel)
    if len(occ) >= 3:  # 2, 4, 8 waves per SIMD in the sweep's order (65 536, 131 072, 262 144 arenas)
        plateau = max(occ[1], occ[2])
        res.update({"rate_by_waves_per_simd": {"2": occ[0], "4": occ[1], "8": occ[2]},
                    "issue_frac": round(occ[0] / plateau, 3)})
        res["sources"]["occupancy"] = os.path.relpath(occ_path, ROOT)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "footsies_gym_amd", "libfootsies.so"))
    ap.add_argument("--kernel", default="_ZN3fsk8k_step_nILi0ELi0EEEvNS_10StepParamsE")
    ap.add_argument("--probe", default=os.path.join(ROOT, "profiles", "r03_valu_probe.json"))
    ap.add_argument("--sq", default=os.path.join(ROOT, "profiles", "r03a_sq.json"))
    ap.add_argument("--sq-kernel", default="fsk::k_step_n<0, 0>", help="the kernel's name in the SQ summary")
    ap.add_argument("--occupancy", default=os.path.join(ROOT, "profiles", "r03_occupancy.txt"))
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    res = model(a.lib, a.kernel, a.probe, a.sq, a.sq_kernel, a.occupancy)
    print(json.dumps(res, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
