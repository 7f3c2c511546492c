#!/usr/bin/env python3
"""Check the shipped code objects for the round-3 fault class:
an LDS read issued from inline asm (ds_read_b128 with a hand-counted lgkmcnt) still
in flight into a register the compiler reuses in the epilogue.

Extracts the gfx950 code objects from build/libbert.so (clang offload bundles in
.hip_fatbin), disassembles every GEMM / attention kernel, and checks that on every
straight-line path from the last LDS read of the K loop (the last one ahead of the
last MFMA before the first store) to the first global / buffer store of the epilogue
there is an `s_waitcnt` with lgkmcnt(0).  Usage:
  scripts/check_drain.py [libbert.so]        -> prints one line per kernel, rc 1 on a miss
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(so):
    """gfx950 code objects of every offload bundle in the shared library."""
    data = open(so, "rb").read()
    objs = []
    pos = data.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" in triple and size:
                objs.append(data[pos + off:pos + off + size])
        pos = data.find(MAGIC, pos + 1)
    return objs


def kernels(so):
    """{symbol: [instruction lines]} of every kernel in the library's device code."""
    out = {}
    with tempfile.TemporaryDirectory() as d:
        for i, co in enumerate(code_objects(so)):
            f = os.path.join(d, f"co{i}.o")
            open(f, "wb").write(co)
            txt = subprocess.run([OBJDUMP, "-d", f], capture_output=True, text=True, check=True).stdout
            cur = None
            for line in txt.splitlines():
                m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
                if m:
                    cur = m.group(1)
                    out[cur] = []
                elif cur and line.startswith("\t"):
                    ins = line.strip().split("//")[0].strip()
                    if ins:
                        out[cur].append(ins)
    return out


def lgkm_zero(ins):
    return ins.startswith("s_waitcnt") and ("lgkmcnt(0)" in ins or re.fullmatch(r"s_waitcnt\s+0", ins) is not None)


def check(body):
    """None if the K loop's last LDS read is drained by an lgkmcnt(0) wait placed after
    it and before the first store, else a description of the miss.  The K loop's reads
    (the asm ones among them) all feed MFMAs, so they come before the last MFMA ahead of
    the first store; LDS reads the compiler schedules after that MFMA are the
    epilogue's own (bias, LN parameters, row statistics), which hipcc waits for itself."""
    first_store = next((i for i, s in enumerate(body) if re.match(r"(global|buffer)_store", s)), None)
    if first_store is None:
        return None
    last_mfma = None
    for i in range(first_store):
        if "mfma" in body[i]:
            last_mfma = i
    last_read = None
    for i in range(last_mfma if last_mfma is not None else first_store):
        if body[i].startswith("ds_read"):
            last_read = i
    if last_read is None:
        return None
    if any(lgkm_zero(s) for s in body[last_read + 1:first_store]):
        return None
    return f"ds_read at {last_read} reaches the store at {first_store} without lgkmcnt(0)"


def main():
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "build", "libbert.so")
    ks = kernels(so)
    bad = 0
    n = 0
    for name, body in sorted(ks.items()):
        if "gemmz_kernel" not in name and "attention" not in name:
            continue
        n += 1
        r = check(body)
        if r:
            bad += 1
            print("MISS", name, r)
    print(f"{n} GEMM / attention kernels checked, {bad} without the drain")
    return 1 if bad or n == 0 else 0


if __name__ == "__main__":
    sys.exit(main())
