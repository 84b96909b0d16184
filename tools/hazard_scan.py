#!/usr/bin/env python3
"""Scan compiler-emitted gfx950 assembly (hipcc --cuda-device-only -S) for VALU pipeline hazards that the
compiler's hazard recognizer does not cover across inline-asm boundaries.

The recognizer inserts wait states for hazards between instructions it generated itself, but an inline
asm block is opaque to most of its checks: a v_exp_f32 the compiler emits right before an asm block that
reads the exp's result gets no wait state (the gfx940/gfx950 "trans forwarding" hazard needs one), and an
asm block's first instruction may be a DPP / permlane read of a VGPR the compiler wrote on the previous
cycle.  Each finding is printed with the kernel, line, producer and consumer.  Straight-line
approximation: wait states are counted along the text (s_nop N = N + 1, any other instruction = 1);
a label resets nothing (conservative: a hazard across a branch target is still reported).

  python3 tools/hazard_scan.py /tmp/isa/bwd_pair.s
"""
import re
import sys

TRANS = re.compile(r"^v_(exp|log|rcp|rsq|sqrt|sin|cos|rcp_iflag)_(f32|f16|legacy_f32)")
VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text):
    out = set()
    for m in VREG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def split_ops(line):
    parts = line.strip().split(None, 1)
    mnem = parts[0]
    ops = parts[1] if len(parts) > 1 else ""
    ops = ops.split(";")[0]
    fields = [f.strip() for f in ops.split(",")]
    return mnem, fields


def main(path, window=2):
    insts = []   # (lineno, mnem, dst_regs, src_regs, in_asm, text)
    in_asm = False
    kernel = None
    findings = []
    with open(path) as f:
        lines = f.readlines()
    for i, raw in enumerate(lines, 1):
        s = raw.strip()
        if s.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if re.match(r"^_Z\w+:", s) and not raw[0].isspace():
            kernel = s.split(":")[0]
            insts.append(None)
            continue
        if s.endswith(":") and s.startswith(".LBB"):
            insts.append(("label", s[:-1]))
            continue
        if not s or s.startswith((";", ".", "//")) or s.endswith(":"):
            continue
        mnem, fields = split_ops(s)
        if not re.match(r"^[sv]_|^global_|^buffer_|^ds_|^flat_|^scratch_", mnem):
            continue
        dst, src = set(), set()
        if mnem.startswith("v_") and fields and fields[0]:
            dst = regs(fields[0])
            src = set().union(*[regs(x) for x in fields[1:]]) if len(fields) > 1 else set()
            if "permlane" in mnem and "swap" in mnem:   # both operands read and written
                src |= dst | (regs(fields[1]) if len(fields) > 1 else set())
                dst = dst | (regs(fields[1]) if len(fields) > 1 else set())
        insts.append((i, mnem, dst, src, in_asm, s, kernel))
    # control flow: the instructions before every branch to a label also precede that label's first
    # instructions (loop back edges, jumps over blocks).  Each predecessor path is checked separately.
    preds = {}
    for idx, it in enumerate(insts):
        if it is None or it[0] == "label":
            continue
        m = re.match(r"^s_(cbranch_\w+|branch)$", it[1])
        if m:
            tgt = it[5].split()[1]
            preds.setdefault(tgt, []).append(idx)
    label_at = {it[1]: i for i, it in enumerate(insts) if it is not None and it[0] == "label"}

    def walk_back(j, ws, src, cons, out, depth=0):
        """From instruction index j backwards (ws wait states already between), find the producer of src."""
        while j >= 0 and ws < 3:
            p = insts[j]
            if p is None:
                return
            if p[0] == "label":
                for b in preds.get(p[1], []):   # a jump into this label: that path's tail
                    if depth < 2:
                        walk_back(b - 1, ws + 1, src, cons, out, depth + 1)
                j -= 1
                continue
            pln, pm, pdst, psrc, asm_p, ptext, _ = p
            if re.match(r"^s_(branch|cbranch_\w+)$", pm) and j != cons - 1:
                if pm == "s_branch":    # unconditional: the fall-through path does not reach here
                    return
            if pm.startswith("s_nop"):
                try:
                    ws += int(ptext.split()[1], 0) + 1
                except Exception:
                    ws += 1
                j -= 1
                continue
            if pm.startswith("v_") and pdst and (pdst & src):
                out.append((p, ws))
                return
            ws += 1
            j -= 1

    for idx, it in enumerate(insts):
        if it is None or it[0] == "label":
            continue
        ln, mnem, dst, src, asm_c, text, kern = it
        if not mnem.startswith("v_"):
            continue
        # gfx950 packed fp32 with op_sel[src] = 1 (the LOW result reading a source's HIGH half): from our
        # inline asm it gave wrong low halves in lanes 48-63 under concurrent load; the
        # compiler emits it too in a few places outside the scan kernels (conv1d_fwd, SS2D merge_bwd)
        m_os = re.search(r"op_sel:\[([01,]+)\]", text)
        if re.match(r"^v_pk_(fma|mul|add)_f32", mnem) and m_os and "1" in m_os.group(1):
            findings.append(("pk_f32 op_sel hi->lo", kern, ln, text, ln, text, asm_c, asm_c))
        is_dpp = "_dpp" in mnem or "row_" in text or "quad_perm" in text
        is_perm = "permlane" in mnem
        is_trans_c = bool(TRANS.match(mnem))
        prods = []
        walk_back(idx - 1, 0, src, idx, prods)
        for p, ws in prods:
            pln, pm, pdst, psrc, asm_p, ptext, _ = p
            if True:
                # gfx940 / gfx950 trans forwarding: non-trans VALU reading a trans result needs 1 wait state
                if TRANS.match(pm) and not is_trans_c and ws < 1:
                    findings.append(("trans->valu", kern, pln, ptext, ln, text, asm_p, asm_c))
                # VALU write -> DPP read of that VGPR: 2 wait states
                if is_dpp and ws < 2:
                    findings.append(("valu->dpp", kern, pln, ptext, ln, text, asm_p, asm_c))
                # gfx950: a packed-fp32 result (v_pk_fma / mul / add_f32) read by the next VALU needs 1 wait state
                if re.match(r"^v_pk_(fma|mul|add)_f32", pm) and ws < 1:
                    findings.append(("pk_f32->valu", kern, pln, ptext, ln, text, asm_p, asm_c))
                if is_perm and ws < 2:
                    findings.append(("valu->permlane", kern, pln, ptext, ln, text, asm_p, asm_c))
    return findings


def report(findings):
    seen = {}
    for f in findings:
        kind, kern, pln, ptext, ln, text, asm_p, asm_c = f
        key = (kind, kern)
        seen.setdefault(key, []).append(f)
    for (kind, kern), fs in sorted(seen.items()):
        print(f"== {kind} in {kern[:90]}: {len(fs)} sites")
        for f in fs[:6]:
            _, _, pln, ptext, ln, text, asm_p, asm_c = f
            print(f"   L{pln}{' [asm]' if asm_p else ''}: {ptext}\n   L{ln}{' [asm]' if asm_c else ''}: {text}")
    if not findings:
        print("no findings")


if __name__ == "__main__":
    report(main(sys.argv[1]))
