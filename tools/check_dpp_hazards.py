#!/usr/bin/env python3
"""Static check of the VALU-write -> DPP-read hazard in libqpb's gfx950 code.

gfx950 needs two wait states between a VALU instruction that writes a VGPR and
a DPP instruction that reads that VGPR as its DPP (src0) operand.  hipcc pads
the DPP moves it generates itself, but not the hand-written v_fmac_f64_dpp of
fmac_bc (csrc/qpb_common.h): there the ordering points of the source are the
only guarantee, and a compiler update could break it silently.

The check disassembles the device code object of every build/*.o with
llvm-objdump, and for every DPP instruction walks back through the
instructions that precede it (following every branch into the block it sits
in) until two wait states are covered (each instruction counts one, s_nop N
counts N + 1); a VALU instruction on that path that writes a register of the
DPP operand is a violation.

usage: check_dpp_hazards.py [build dir]   (exit 1 and a listing on violations)
"""
import glob
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
INSN = re.compile(r"^\s+([a-z_0-9]+)(?:\s+(.*?))?\s*//\s*([0-9A-Fa-f]+):\s*([0-9A-Fa-f ]+)$")
BRANCH = re.compile(r"^s_(c?branch\w*)$")


def vregs(op):
    """set of VGPR numbers named by an operand string (v7, v[4:5])"""
    op = op.strip()
    m = re.match(r"^-?\|?v\[(\d+):(\d+)\]", op)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"^-?\|?v(\d+)\b", op)
    if m:
        return {int(m.group(1))}
    return set()


def split_ops(s):
    if not s:
        return []
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur:
        out.append(cur)
    return [o.strip() for o in out]


def parse(text):
    """-> list of functions, each a list of (addr, mnemonic, operands-string)"""
    funcs, cur = [], None
    for line in text.splitlines():
        if re.match(r"^[0-9a-f]+ <.*>:$", line):
            cur = []
            funcs.append((line, cur))
            continue
        m = INSN.match(line)
        if m and cur is not None:
            ops = m.group(2) or ""
            words = m.group(4).split()
            cur.append((int(m.group(3), 16), m.group(1), ops, len(words) * 4))
    return funcs


def check_function(insns):
    idx = {a: i for i, (a, _, _, _) in enumerate(insns)}
    preds = {}  # instruction index -> list of branch instruction indices jumping to it
    for i, (a, mn, ops, size) in enumerate(insns):
        if BRANCH.match(mn):
            m = re.match(r"^(-?\d+)", ops.split()[0] if ops else "")
            if not m:
                continue
            tgt = a + 4 + 4 * int(m.group(1))
            if tgt in idx:
                preds.setdefault(idx[tgt], []).append(i)
    bad = []
    for i, (a, mn, ops, _) in enumerate(insns):
        if not (mn.startswith("v_") and mn.endswith("_dpp")):
            continue
        o = split_ops(ops.split(" row_")[0].split(" quad_perm")[0])
        if len(o) < 2:
            continue
        src = vregs(o[1])
        if not src:
            continue
        # walk back along every path until 2 wait states are covered
        stack = [(i, 0)]
        seen = set()
        while stack:
            j, ws = stack.pop()
            if (j, ws) in seen:
                continue
            seen.add((j, ws))
            if ws >= 2:
                continue
            fall = [j - 1] if j >= 1 and insns[j - 1][1] not in ("s_branch", "s_endpgm", "s_setpc_b64") else []
            for k in fall + preds.get(j, []):
                if k < 0:
                    continue
                kmn, kops = insns[k][1], insns[k][2]
                if kmn == "s_nop":
                    n = int(kops.split()[0], 0) if kops else 0
                    stack.append((k, ws + n + 1))
                    continue
                if BRANCH.match(kmn):  # a branch is not a wait state; look past it
                    stack.append((k, ws))
                    continue
                if kmn.startswith("v_") and not kmn.startswith(("v_cmp", "v_readlane", "v_readfirstlane")):
                    dst = vregs(split_ops(kops)[0]) if kops else set()
                    if dst & src:
                        bad.append((a, mn, ops, insns[k][0], kmn, kops))
                        continue
                stack.append((k, ws + 1))
    return bad


def main(build):
    objs = sorted(glob.glob(os.path.join(build, "*.o")))
    total_dpp, violations = 0, []
    with tempfile.TemporaryDirectory() as td:
        for o in objs:
            tmp = os.path.join(td, os.path.basename(o))
            shutil.copy(o, tmp)
            subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", tmp], cwd=td, capture_output=True)
            for co in glob.glob(tmp + ".*gfx950*"):
                text = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], capture_output=True,
                                      text=True).stdout
                for name, insns in parse(text):
                    total_dpp += sum(1 for _, mn, _, _ in insns if mn.startswith("v_") and mn.endswith("_dpp"))
                    for v in check_function(insns):
                        violations.append((os.path.basename(o), name, v))
    for o, name, (a, mn, ops, ka, kmn, kops) in violations:
        print(f"{o} {name} {a:#x}: {mn} {ops}  <- {ka:#x}: {kmn} {kops}")
    print(f"{len(objs)} objects, {total_dpp} DPP instructions, {len(violations)} hazards")
    return 1 if violations else 0


if __name__ == "__main__":
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(here, "embedded-qp-solver_amd", "build")))
