"""Build-time ISA check of the descent's asm load (OCH_ASM_LOAD, och_kernels.hip).

The grid and bounce kernels issue the child's slot-word load into the ray's
current-node register `cur` by inline asm, outside the compiler's waitcnt
view, and wait for it with an explicit `s_waitcnt vmcnt(0)` that takes `cur`
as an operand (nothing else guarantees the compiler never touches
`cur` while the load is in flight).  This compiles the kernels to assembly
with the product's flags and checks, in every function that issues the load
(the per-node skip's box load is the compiler's own and needs no check):
  1. the first vmcnt(0) wait on every path from a load, if it is cur's own
     wait, names the register the load wrote (a compiler copy of cur at a
     join would make the wait hand a stale register to the next PUSH);
  2. on every control-flow path from a load to the next vmcnt(0) wait, no
     instruction reads that register before an instruction on the same path
     has written it.  Such a read would take the word before the load lands
     (a copy, a spill, a full-wave select).  Writes there are allowed: they are
     the STEP phase's temporaries in lanes that issued no load (exec-masked,
     so the load's return and they never meet, och_kernels.hip OCH_ASM_LOAD).
  3. in every function, a lane mask (vcc or an SGPR pair) written by a VALU
     compare is read as a lane mask (v_cndmask, a carry-in) no sooner than 2
     wait states later (instructions or s_nop states in between, within a basic
     block; a carry-out read as the next carry-in, the 64-bit add chain, is not
     this hazard).  The compiler keeps that distance in
     its own code (its minimum over these kernels is 2); the check holds the
     hand-placed VALU of the descent's child index (ray_push_descend) to it.
  4. every traversal kernel (k_trace_grid, k_trace_bounce) admits 8 waves per
     SIMD by its SGPR and VGPR counts (above 80 SGPRs a SIMD takes 7, although
     the compiler's occupancy note still says 8).
  5. no grid kernel spills SGPRs to VGPR lanes (the config-5 kernels' spills are
     counted in the summary).
Exit status 0 and a one-line summary when every kernel passes; 1 with the
offending instruction otherwise.  Run by the csrc Makefile (`make isa-check`),
__graft_entry__.build() and tests/test_isa_check.py.

Usage: python tools/isa_check.py [--source och_kernels.hip] [--asm file.s] [-D NAME=VALUE ...]
"""
from __future__ import annotations

import argparse
import json
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "octree_ray_tracing_amd" / "csrc"
HIPCC = "/opt/rocm/bin/hipcc"
# the product's flags (csrc/Makefile FLAGS + DEVFLAGS), device code only
FLAGS = ["-std=c++17", "-O3", "-ffp-contract=off", "-fno-fast-math", "--offload-arch=gfx950",
         "-fno-gpu-flush-denormals-to-zero", "-munsafe-fp-atomics", "--cuda-device-only", "-S"]

REG_RE = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")
LABEL_RE = re.compile(r"^(\.LBB\d+_\d+|[A-Za-z_.$][\w.$]*):")
# instructions without a VGPR destination: every vector operand is a source
NO_VDST = re.compile(r"^(s_|v_cmp|v_cmpx|v_readfirstlane|v_readlane|global_store|buffer_store|flat_store|"
                     r"scratch_store|ds_write|ds_store|exp\b|global_atomic(?!.*\bsc0\b)|ds_add_u32|ds_gws)")
# instructions whose destination is also read (partial writes)
PARTIAL_DST = re.compile(r"(_sdwa|_d16|_hi\b|_dpp\b|v_writelane|v_mac_|v_fmac_)")


def compile_asm(source: Path, defines: list[str]) -> str:
    with tempfile.TemporaryDirectory() as d:
        out = Path(d) / "k.s"
        cmd = [HIPCC, *FLAGS, *[f"-D{x}" for x in defines], str(source), "-o", str(out)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise SystemExit(f"isa_check: compile failed:\n{r.stderr[-2000:]}")
        return out.read_text()


def regs(text: str) -> set[int]:
    out = set()
    for m in REG_RE.finditer(text):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def split_operands(ins: str):
    """(mnemonic, [operand strings]) of one instruction, comment stripped."""
    body = ins.split(";")[0].split("//")[0].strip()
    if not body:
        return "", []
    parts = body.split(None, 1)
    mn = parts[0]
    ops = [o.strip() for o in re.split(r",(?![^\[]*\])", parts[1])] if len(parts) > 1 else []
    return mn, ops


def reads_writes(ins: str):
    """(VGPRs read, VGPRs fully written) by one instruction."""
    mn, ops = split_operands(ins)
    if not mn or not ops:
        return set(), set()
    if NO_VDST.match(mn):
        return set().union(*(regs(o) for o in ops)), set()
    dst = regs(ops[0])
    src = set().union(*(regs(o) for o in ops[1:])) if len(ops) > 1 else set()
    if PARTIAL_DST.search(mn):
        src |= dst
    return src, dst


def functions(asm: str):
    """{name: [lines]} of every function body in the assembly text."""
    out, cur, name = {}, None, None
    for line in asm.splitlines():
        if cur is None:
            m = re.match(r"^([_A-Za-z][\w.$]*):\s*(;.*)?$", line)
            if m and not line.startswith(".L"):
                name, cur = m.group(1), []
            continue
        if re.match(r"^\.Lfunc_end\d+:", line):
            out[name] = cur
            cur = None
            continue
        cur.append(line)
    return out


def check_function(name: str, lines: list[str]):
    """Problems of one function (empty list = passes), and its load count."""
    ins, labels = [], {}
    for line in lines:
        m = LABEL_RE.match(line)
        if m:
            labels[m.group(1)] = len(ins)
            continue
        t = line.strip()
        if not t or t.startswith((".", ";")):
            continue
        ins.append(t)
    # the descent's asm loads of the child's word into cur (och_cur_load)
    loads = [i for i, t in enumerate(ins) if "och_cur_load" in t]
    if not loads:
        return [], 0
    problems = []

    def successors(pc: int):
        mn, ops = split_operands(ins[pc])
        if mn == "s_branch":
            return [labels[ops[0]]] if ops and ops[0] in labels else []
        if mn.startswith("s_cbranch"):
            tgt = [labels[ops[0]]] if ops and ops[0] in labels else []
            return tgt + [pc + 1]
        if mn in ("s_endpgm", "s_setpc_b64", "s_trap"):
            return []
        return [pc + 1]

    for start in loads:
        creg_text = split_operands(ins[start])[1][0]
        creg = regs(creg_text)
        seen = set()
        stack = [(start + 1, False)]
        while stack:
            pc, written = stack.pop()
            if pc >= len(ins) or (pc, written) in seen:
                continue
            seen.add((pc, written))
            t = ins[pc]
            mn, _ = split_operands(t)
            if mn in ("s_swappc_b64", "s_setpc_b64"):
                problems.append(f"{name}: call with a cur load in flight: {t}")
                continue
            if mn == "s_waitcnt" and "vmcnt(0)" in t:
                # the load has landed; if this is cur's own wait, it must hand
                # on the register the load wrote (no copy of cur in between)
                named = t.split("och_cur_wait", 1)[1].split() if "och_cur_wait" in t else None
                if named is not None and (not named or named[0] != creg_text):
                    problems.append(f"{name}: the load into {creg_text} (instruction {start}) is waited for as "
                                    f"{' '.join(named)}: the register was copied while in flight")
                continue
            rd, wr = reads_writes(t)
            if rd & creg and not written:
                problems.append(f"{name}: reads {creg_text} while the asm load may be in flight "
                                f"(load at instruction {start}): {t}")
                continue
            if wr & creg:
                written = True
            for nxt in successors(pc):
                stack.append((nxt, written))
    return problems, len(loads)


MASK_READ_E32 = ("v_cndmask_b32_e32", "v_addc_co_u32_e32", "v_subb_co_u32_e32", "v_subbrev_co_u32_e32")
MASK_READ_E64 = ("v_cndmask_b32_e64", "v_addc_co_u32_e64", "v_subb_co_u32_e64", "v_subbrev_co_u32_e64")
CARRY_WRITE = re.compile(r"^v_(add|sub|subrev|addc|subb|subbrev)_co_u32_(e32|e64)$")
MASK_WAIT_STATES = 2


def check_mask_hazards(name: str, lines: list[str]) -> list[str]:
    """Check 3: VALU lane-mask writes and their reads as lane masks."""
    problems, last, pos = [], {}, 0
    for line in lines:
        t = line.split(";")[0].strip()
        if not t or t.startswith("."):
            if LABEL_RE.match(t):
                last = {}
            continue
        if LABEL_RE.match(t):
            last = {}
            continue
        mn, ops = split_operands(t)
        if mn == "s_nop":
            pos += int(ops[0], 0) + 1
            continue
        read = "vcc" if mn in MASK_READ_E32 else (ops[-1] if mn in MASK_READ_E64 and ops else None)
        if read in last and last[read] is not None and pos - last[read] < MASK_WAIT_STATES:
            problems.append(f"{name}: {t} reads the lane mask {read} {pos - last[read]} wait state(s) after "
                            f"a VALU wrote it (needs {MASK_WAIT_STATES})")
        pos += 1
        if mn.startswith("v_cmp_"):
            dst = "vcc" if mn.endswith(("_e32", "_sdwa")) else (ops[0] if ops else None)
            if dst:
                last[dst] = pos
        elif CARRY_WRITE.match(mn):
            dst = "vcc" if mn.endswith("_e32") else (ops[1] if len(ops) > 1 else None)
            if dst:
                last[dst] = None               # a carry-out: not a compare's mask
        elif mn.startswith("s_") and ops and ops[0] in last:
            del last[ops[0]]                   # a scalar write replaces the VALU's
    return problems


RENDER_KERNEL = "k_trace_gridINS0_12CameraSourceENS0_9FrameSinkELi1ELb0"   # the bench's render launch


def walk_loop_counts(lines: list[str]):
    """Static VALU / SALU of each walk loop (a loop holding the descent's asm
    load) of one function: from its header to the descent's branch back to the
    latch, plus the latch.  A list of (valu, salu, reads the stack's idx plane);
    empty when the layout is not recognised."""
    ins = [l.split(";")[0].rstrip() if not l.lstrip().startswith(".LBB") else l for l in lines]
    pos = {m.group(1): i for i, l in enumerate(ins) if (m := re.match(r"^(\.LBB\d+_\d+):", l.strip()))}
    loops = []
    for i, l in enumerate(lines):
        if "Inner Loop Header: Depth=1" not in l:
            continue
        for k in range(i + 1, len(lines)):
            m = re.match(r"\s*s_branch\s+(\.LBB\d+_\d+)", lines[k])
            if m and pos.get(m.group(1), len(lines)) < i:
                body = lines[i:k + 1] + lines[pos[m.group(1)]:i]
                if any("och_cur_load" in b for b in body):
                    valu = sum(1 for b in body if re.match(r"\s*v_", b))
                    salu = sum(1 for b in body if re.match(r"\s*s_", b)
                               and not re.match(r"\s*s_(nop|waitcnt|cbranch|branch)", b))
                    loops.append((valu, salu, any(re.match(r"\s*ds_read_u8", b) for b in body)))
                break
    return loops


def kernel_resources(asm: str):
    """{kernel name: (sgpr_count, vgpr_count)} from the code object's metadata."""
    names = [(m.start(), m.group(1)) for m in re.finditer(r"^\s+\.name:\s+(\S+)", asm, re.M)]
    out = {}
    for i, (pos, name) in enumerate(names):
        end = names[i + 1][0] if i + 1 < len(names) else len(asm)
        blk = asm[pos:end]
        sg = re.search(r"\.sgpr_count:\s+(\d+)", blk)
        vg = re.search(r"\.vgpr_count:\s+(\d+)", blk)
        if sg and vg:
            out[name] = (int(sg.group(1)), int(vg.group(1)))
    return out


def waves_per_simd(sgpr: int, vgpr: int) -> int:
    """Waves a SIMD admits for these registers (MI355X_MICROARCH.md: residency,
    register files): SGPRs in granules of 16 plus 16 from an 800-entry file,
    VGPRs in granules of 8 from 512, at most 8."""
    by_sgpr = 800 // (((sgpr + 15) // 16) * 16 + 16)
    by_vgpr = 512 // (((vgpr + 7) // 8) * 8)
    return min(8, by_sgpr, by_vgpr)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--source", default=str(CSRC / "och_kernels.hip"))
    ap.add_argument("--asm", default=None, help="check this assembly file instead of compiling")
    ap.add_argument("-D", dest="defines", action="append", default=[])
    a = ap.parse_args(argv)
    asm = Path(a.asm).read_text() if a.asm else compile_asm(Path(a.source), a.defines)
    fns = functions(asm)
    checked, problems, loads = [], [], 0
    for name, lines in fns.items():
        p, n = check_function(name, lines)
        if n:
            checked.append(name)
            loads += n
        problems += p
        problems += check_mask_hazards(name, lines)
    want = ("k_trace_grid", "k_trace_bounce")
    missing = [w for w in want if not any(w in c for c in checked)]
    asm_on = "och_cur_load" in asm
    summary = {"functions": len(fns), "checked": len(checked), "asm_loads": loads, "problems": len(problems),
               "asm_load_enabled": asm_on}
    render = [n for n in fns if RENDER_KERNEL in n]
    loops = walk_loop_counts(fns[render[0]]) if render else []
    if loops:
        # the walk that reads idx from the stack (every wave whose rays start inside
        # the root) first; the rebuilding walk of the other waves beside it
        loops.sort(key=lambda t: not t[2])
        summary["render_loop_valu"], summary["render_loop_salu"] = loops[0][:2]
        summary["render_loops"] = [{"valu": v, "salu": s_, "idx_plane": ip} for v, s_, ip in loops]
    if asm_on and missing:
        problems.append(f"no asm load found in {missing}")
    # 4. the traversal kernels keep 8 waves per SIMD (82 SGPRs admitted 7 and cost
    #    5 % sustained); the compiler's own occupancy note says 8 there
    res = kernel_resources(asm)
    occ = {n: waves_per_simd(*r) for n, r in res.items() if "k_trace_grid" in n or "k_trace_bounce" in n}
    if render and render[0] in res:
        summary["render_sgpr"], summary["render_vgpr"] = res[render[0]]
    summary["traversal_waves_per_simd"] = min(occ.values()) if occ else None
    for n, w in occ.items():
        if w < 8:
            problems.append(f"{n}: {res[n][0]} SGPRs / {res[n][1]} VGPRs admit {w} waves per SIMD, not 8")
    # 5. no grid kernel spills SGPRs to VGPR lanes: under the 80-SGPR cap the
    #    compiler spills rather than drop to 7 waves, and a spill reloaded in every
    #    wave cost the split kernel 2 %.  The config-5 kernels
    #    spill in their per-ray setup (counted, not refused).
    spills = {n: sum(1 for l in lines if re.match(r"\s*v_(writelane|readlane)_b32", l))
              for n, lines in fns.items() if "k_trace_grid" in n or "k_trace_bounce" in n}
    summary["grid_spill_lanes"] = sum(v for n, v in spills.items() if "k_trace_grid" in n)
    summary["bounce_spill_lanes"] = sum(v for n, v in spills.items() if "k_trace_bounce" in n)
    for n, v in spills.items():
        if v and "k_trace_grid" in n:
            problems.append(f"{n}: {v} SGPR spill lanes (v_writelane / v_readlane)")
    if problems:
        print("isa_check: FAILED " + json.dumps(summary))
        for p in problems[:20]:
            print("  " + p)
        return 1
    print("isa_check: ok " + json.dumps(summary))
    return 0


if __name__ == "__main__":
    sys.exit(main())
