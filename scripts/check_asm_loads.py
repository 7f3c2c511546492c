#!/usr/bin/env python3
"""Check the shipped code objects for the asm-load hazard of attention_pp: its Q rows
are loaded by inline-asm global_load_dwordx4 (invisible to hipcc's waitcnt pass) and
retired by one s_waitcnt tied to the registers.  Between each load's issue and that
wait no instruction may read or write the load's destination registers (hipcc once
copied them in front of per-branch waits, before the data landed), and no later
load of the group may use a pending destination as its address.
  scripts/check_asm_loads.py [libbert.so]   -> one line per kernel, rc 1 on a hit"""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from check_drain import OBJDUMP, ROOT, code_objects  # noqa: E402


def kernels(so):
    out = {}
    for co in code_objects(so):
        with tempfile.NamedTemporaryFile(suffix=".o") as f:
            f.write(co)
            f.flush()
            txt = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", f.name], capture_output=True, text=True).stdout
        for fn in re.split(r"\n(?=[0-9a-f]{16} <)", txt):
            head = fn.split("\n", 1)[0]
            if "attention_pp" in head:
                out[head] = [re.sub(r"\s+//.*", "", ln.strip()) for ln in fn.split("\n")]
    return out


def regs(op):
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", op)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"v(\d+)", op)
    return {int(m.group(1))} if m else set()


def check(lines):
    loads = [i for i, ln in enumerate(lines) if ln.startswith("global_load_dwordx4 ")]
    if len(loads) < 4:
        return "no asm Q loads found"
    wait = next(i for i, ln in enumerate(lines) if i > loads[3] and ln.startswith("s_waitcnt") and "vmcnt" in ln)
    pending = set()
    for i in range(loads[0], wait):
        ops = [regs(o) for o in re.findall(r"v\[\d+:\d+\]|v\d+", lines[i])]
        if lines[i].startswith("global_load_dwordx4 "):
            if len(ops) > 1 and ops[1] & pending:
                return f"line {i}: address reads a pending destination: {lines[i]}"
            pending |= ops[0]
            continue
        for r in ops:
            if r & pending:
                return f"line {i}: touches a pending Q register: {lines[i]}"
    return None


def main():
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "build", "libbert.so")
    ks = kernels(so)
    bad = 0
    for head, lines in sorted(ks.items()):
        err = check(lines)
        print(("FAIL " + err) if err else "ok  ", head.split("<", 1)[1][:70])
        bad += err is not None
    if not ks:
        print("no attention_pp kernels found")
        return 1
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
