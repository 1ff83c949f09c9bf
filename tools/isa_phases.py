#!/usr/bin/env python3
"""Attribute the fused step kernel's main-loop instructions to the C# phases they restate.

  python tools/isa_phases.py [--kernel _ZN3fsk8k_step_nILi0ELi0EEEvNS_10StepParamsE]
                             [--src footsies_gym_amd/csrc/fs_kernels.hip] [--json profiles/r04_isa_phases.json]

fs_kernels.hip is compiled for gfx950 with the library's own flags (footsies_gym_amd/build.py)
plus -gline-tables-only, which adds line tables with inlining records and leaves the code alone
(checked here: the kernel's mnemonic sequence must equal the one in the built libfootsies.so).
Every instruction of the main loop (the backward branch spanning the most instructions, two
ticks of the row loop; tools/issue_model.main_loop) is symbolized with its full inline chain
(llvm-symbolizer --inlines) and charged to the outermost function called from env_step (the
tick), or to the env_step / step_body source line range it sits on when the tick body itself
holds it.  Functions map to phases (PHASES below, with the C# each one restates).  Phases that
run only on rare lanes -- a landed hit (NotifyDamaged), the KO / reset burst, the terminal
record -- are reported apart from the common path, whose per-tick counts are what
profiles/*_sq.json measures (SQ_INSTS_VALU etc. per wave-tick).
"""
import argparse
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from footsies_gym_amd import build as B  # noqa: E402
import issue_model as IM  # noqa: E402

LLVM = "/opt/rocm/lib/llvm/bin"

# function (as llvm-symbolizer --functions=short prints it, template arguments stripped) -> phase
PHASES = {
    "update_input": "UpdateInput + dash / charge parsers (F:172-188, 569-635)",
    "increment_action_frame": "IncrementActionFrame (F:140-166)",
    "frame_record": "UpdateActionRequest: record index of (action, frame) (AD:87-168)",
    "request_sel": "UpdateActionRequest: request-table index (F:201-286)",
    "apply_request": "UpdateActionRequest / RequestAction / SetCurrentAction apply (F:472-510, 546-563)",
    "update_action_request": "UpdateActionRequest: request-table read (F:201-286)",
    "frame_rec": "UpdateBoxes: frame record read (F:671-719)",
    "update_movement": "UpdateMovement (F:291-319)",
    "update_boxes": "UpdateBoxes (F:671-697)",
    "push_character_vs_character": "UpdatePushCharacterVsCharacter (BC:483-501)",
    "push_character_vs_background": "UpdatePushCharacterVsBackground (BC:503-519)",
    "apply_position_change": "ApplyPositionChange (F:331-350)",
    "hitbox_hurtbox_collision": "UpdateHitboxHurtboxCollision (BC:521-591)",
    "box_x_overlaps": "UpdateHitboxHurtboxCollision: BoxBase.Overlaps x (F:17-25)",
    "notify_damaged": "NotifyDamaged (F:357-398) [rare]",
    "attack_info": "NotifyDamaged: AttackData select [rare]",
    "write_main": "outputs: EnvironmentState / obs / info (BC:449-468, FE:336-380)",
    "write_obs": "outputs: EnvironmentState / obs / info (BC:449-468, FE:336-380)",
    "write_final": "outputs: terminal record (FE same-step reset) [rare]",
    "st_off": "outputs: EnvironmentState / obs / info (BC:449-468, FE:336-380)",
    "reset_burst": "KO -> End -> Intro -> Fight burst (BC:212-345) [rare]",
    "end_tick": "KO -> End -> Intro -> Fight burst (BC:212-345) [rare]",
    "setup_battle_start": "KO -> End -> Intro -> Fight burst (BC:212-345) [rare]",
    "opaque_burst_results": "KO -> End -> Intro -> Fight burst (BC:212-345) [rare]",
    "stand_info": "KO -> End -> Intro -> Fight burst (BC:212-345) [rare]",
    "action_info": "next tick's ActionInfo read (F:140-166 / 472-510 inputs)",
    "settle_w": "action rows: wait for the next tick's row (TrainingRemoteActor input)",
    "row_load": "action rows: load (TrainingRemoteActor input)",
    "prio_slice": "wave priority slice (scheduling, no C# counterpart)",
    "prio_group": "wave priority slice (scheduling, no C# counterpart)",
    "bot_prefetch": "BattleAI (AI:41-403)",
    "bot_next_input": "BattleAI (AI:41-403)",
    "stored_input": "inputs: actor input (BC:383-447)",
}
# env_step's own source lines, by the comment that heads each stretch (found in the source)
ENV_STEP_MARKS = [
    ("the actor inputs of this frame", "inputs: actor input (BC:383-447)"),
    ("RecordInput (BC:593-607)", "RecordInput + frameCount (BC:201-220, 593-607)"),
    ("One LDS round trip for everything", "UpdateBoxes: y-overlap / resolution reads + pair exchange (BC:521-591)"),
    ("the partner's hitbox half-widths", "UpdateHitboxHurtboxCollision (BC:521-591)"),
    ("KO check (BC:212-213) and reward", "KO test + reward flags (BC:212-213, FE:382-405)"),
    ("Only a guard drop or the round's end moves the f64 sums", "dense reward in f64 (FE:388-405) [rare]"),
    ("} else {\n    const uint32_t fl2 = k == 0 ? o_fl : my_fl;", "KO test + reward flags (BC:212-213, FE:382-405)"),
    ("settle_w<WAIT>(next);\n  if (over) {", "action rows: wait for the next tick's row (TrainingRemoteActor input)"),
    ("ChangeRoundState(KO)", "KO -> End -> Intro -> Fight burst (BC:212-345) [rare]"),
    ("TrainingManager.Step -> RequestNextInput", "BattleAI (AI:41-403)"),
    ("if constexpr (PK) {\n    write_packed(L, o.pk_lanes, r, k == 0 ? (uint32_t)L.frame_count : (over",
     "outputs: EnvironmentState / obs / info (BC:449-468, FE:336-380)"),
]
RARE_TAG = "[rare]"
# functions charged wherever they sit in the chain (the rare work nested inside a common phase)
NESTED = {"notify_damaged", "attack_info"}
# small helpers that belong to their caller's phase: charged to the call site's line in env_step
HELPERS = {"xpair", "xp1", "xp2", "fadd", "fsub", "fadd2", "fsub2", "tabs", "bit0_mask", "splat", "sel4",
           "ai_frame_count", "ai_loop_from", "ai_cancel_lo", "ai_cancel_hi"}


def compile_debug(src, out_dir):
    co = os.path.join(out_dir, "k.co")
    subprocess.run([B._hipcc(), "--offload-arch=" + B.ARCH, *B.flags_for(src), "-gline-tables-only", "-I",
                    os.path.join(ROOT, "include"), "--cuda-device-only", "-c", "-o", co, src], check=True)
    dev = os.path.join(out_dir, "k.gfx950.o")
    subprocess.run([LLVM + "/clang-offload-bundler", "--type=o", "--input=" + co,
                    "--targets=hipv4-amdgcn-amd-amdhsa--" + B.ARCH, "--output=" + dev, "--unbundle"], check=True)
    dis = subprocess.run([LLVM + "/llvm-objdump", "-d", "--mcpu=" + B.ARCH, dev], check=True, capture_output=True,
                         text=True).stdout
    return dev, dis


def symbolize(obj, addrs):
    p = subprocess.run([LLVM + "/llvm-symbolizer", "--inlines", "--functions=short", "--obj=" + obj],
                       input="\n".join("0x%x" % a for a in addrs) + "\n", capture_output=True, text=True, check=True)
    chains, cur = [], []
    lines = p.stdout.split("\n")
    i = 0
    while i < len(lines):
        if lines[i] == "":
            if cur:
                chains.append(cur)
                cur = []
            i += 1
            continue
        fn, loc = lines[i], lines[i + 1] if i + 1 < len(lines) else ""
        m = re.match(r".*:(\d+):(\d+)$", loc)
        cur.append((re.sub(r"<.*$", "", fn), int(m.group(1)) if m else 0))
        i += 2
    if cur:
        chains.append(cur)
    assert len(chains) == len(addrs), (len(chains), len(addrs))
    return chains  # innermost first


def line_marks(src_text):
    """env_step's stretches: (first line, phase) from ENV_STEP_MARKS, in source order."""
    start = re.search(r"__device__ __forceinline__ \w+ env_step\(", src_text).start()
    out = []
    for needle, phase in ENV_STEP_MARKS:
        k = src_text.find(needle, start)
        if k < 0:  # (a mark of another revision's tick)
            continue
        out.append((src_text.count("\n", 0, k) + 1, phase))
    return sorted(out)


def kind(mn):
    if mn.startswith("v_mfma"):
        return "mfma"
    if mn.startswith("v_"):
        return "valu"
    if mn.startswith("ds_"):
        return "lds"
    if mn.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if mn.startswith(("s_load", "s_buffer_load", "s_memrealtime", "s_memtime", "s_dcache")):
        return "smem"
    if mn.startswith(("s_cbranch", "s_branch", "s_setpc", "s_swappc")):
        return "branch"
    if mn.startswith(("s_waitcnt", "s_nop", "s_setprio", "s_barrier", "s_sleep", "s_endpgm")):
        return "misc"
    if mn.startswith("s_"):
        return "salu"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="_ZN3fsk8k_step_nILi0ELi0EEEvNS_10StepParamsE")
    ap.add_argument("--src", default=os.path.join(B.CSRC, "fs_kernels.hip"))
    ap.add_argument("--lib", default=B.LIB)
    ap.add_argument("--sq", default=None, help="profiles/*_sq.json with the measured per-wave-tick counts")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    src_text = open(a.src).read()
    with tempfile.TemporaryDirectory() as d:
        obj, dis = compile_debug(a.src, d)
        insts = IM.kernel_insts(dis, "<" + a.kernel + ">")
        assert insts, "kernel %s not found" % a.kernel
        # the debug build must be the same code as the shipped library
        if os.path.exists(a.lib):
            ship = IM.kernel_insts(IM.disassemble(a.lib), "<" + a.kernel + ">")
            same = [x[1] for x in ship] == [x[1] for x in insts]
            assert same, "the -gline-tables-only build differs from %s" % a.lib
        lo, hi = IM.main_loop(insts)
        loop = insts[lo:hi + 1]
        chains = symbolize(obj, [x[0] for x in loop])
    marks = line_marks(src_text)

    def phase_of(chain):
        outer = list(reversed(chain))  # kernel first
        names = [f for f, _ in outer]
        for fn in names:
            if fn in NESTED:
                return PHASES[fn]
        if "env_step" in names:
            k = names.index("env_step")
            if k + 1 < len(outer) and outer[k + 1][0] not in HELPERS:  # inside a function the tick calls
                fn = outer[k + 1][0]
                return PHASES.get(fn, fn)
            line = outer[k][1]
            ph = "env_step (tick head)"
            for first, p in marks:
                if line >= first:
                    ph = p
            return ph
        if "step_body" in names:
            k = names.index("step_body")
            if k + 1 < len(outer):
                fn = outer[k + 1][0]
                return PHASES.get(fn, "loop: " + fn)
            return "loop control (step_body)"
        return "other: " + names[-1]

    per = collections.defaultdict(collections.Counter)
    cls = collections.defaultdict(collections.Counter)  # VALU issue classes (tools/issue_model.classify)
    prev_vcc = False
    for (addr, mn, ops, size), ch in zip(loop, chains):
        ph = phase_of(ch)
        per[ph][kind(mn)] += 1
        if mn.startswith("v_") and not mn.startswith(("v_readfirstlane", "v_readlane", "v_writelane", "v_mfma")):
            cls[ph][IM.classify(mn, ops, size, prev_vcc)] += 1
            prev_vcc = IM.reads_vcc(mn, ops)
    ticks = 2  # the main loop is the row loop unrolled by two ticks
    rows, common, rare = [], collections.Counter(), collections.Counter()
    for ph, c in per.items():
        tot = sum(c.values())
        row = {"phase": ph, "per_tick": {k: v / ticks for k, v in sorted(c.items())}, "total_per_tick": tot / ticks,
               "valu_classes_per_tick": {k: v / ticks for k, v in sorted(cls[ph].items())}, "rare": RARE_TAG in ph}
        rows.append(row)
        (rare if row["rare"] else common).update(c)
    rows.sort(key=lambda r: (r["rare"], -r["per_tick"].get("valu", 0), -r["total_per_tick"]))
    res = {"kernel": a.kernel, "source": os.path.relpath(a.src, ROOT), "flags": "build.py flags_for(fs_kernels.hip) + -gline-tables-only "
           "(same code as the library: mnemonic sequence checked)",
           "loop_instructions": len(loop), "ticks_in_loop": ticks,
           "common_path_per_tick": {k: v / ticks for k, v in sorted(common.items())},
           "rare_paths_per_tick_static": {k: v / ticks for k, v in sorted(rare.items())},
           "phases": rows,
           "note": "static counts of the main loop (two ticks) / 2, charged by inline chain; rare phases run only "
                   "on waves with a hit / KO lane, and the common-path counts are the ones to compare with the "
                   "measured per-wave-tick SQ counters"}
    if a.sq:
        with open(a.sq) as f:
            sq = json.load(f)
        k0 = [k for k in sq.get("kernels", []) if k.get("kernel", "").endswith(a.kernel.split("fsk")[-1][:10]) or True]
        if k0:
            pw = k0[0].get("per_wave_tick", {})
            res["measured_per_wave_tick"] = {"valu": pw.get("SQ_INSTS_VALU"), "salu": pw.get("SQ_INSTS_SALU"),
                                             "lds": pw.get("SQ_INSTS_LDS"), "source": os.path.relpath(a.sq, ROOT)}
    for r in rows:
        vc = r["valu_classes_per_tick"]
        print("%-82s valu %6.1f  salu %5.1f  lds %4.1f  vmem %4.1f  all %6.1f | vopc %4.1f vop3 %5.1f fast %5.1f" % (
            r["phase"][:82], r["per_tick"].get("valu", 0), r["per_tick"].get("salu", 0), r["per_tick"].get("lds", 0),
            r["per_tick"].get("vmem", 0), r["total_per_tick"], vc.get("vopc", 0), vc.get("vop3_op", 0),
            vc.get("fast", 0)))
    print("common path per tick:", res["common_path_per_tick"])
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
