#!/usr/bin/env python3
"""Resolve the frames of a glog-style native backtrace ("@ 0x... (unknown)") against shared libraries
of this container, offline.

A library is mapped page-aligned, so each frame's address modulo 4096 equals its offset in the file
modulo 4096, and frames of ONE library keep their exact distances.  For every candidate library the
script lists the return addresses (the address after each call instruction, from llvm-objdump) and
searches the load base that makes a whole cluster of frames land on return addresses (or, for the
faulting PC, on an instruction).  A base that explains >= 2 frames of a cluster is reported with
the enclosing symbol of every frame.

usage: symbolize_crash.py LOG [LIB ...]"""
import bisect
import re
import subprocess
import sys

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
DEFAULT_LIBS = ["/opt/rocm/lib/libamdhip64.so.7", "/opt/rocm/lib/libhsa-runtime64.so.1",
                "/opt/rocm/lib/librocprofiler-sdk.so.1", "/opt/rocm/lib/rocprofiler-sdk/librocprofiler-sdk-tool.so",
                "/opt/rocm/lib/librocprofiler-register.so.0", "/lib/x86_64-linux-gnu/libc.so.6",
                "/lib/x86_64-linux-gnu/libstdc++.so.6", "/lib/x86_64-linux-gnu/libgcc_s.so.1"]


def disasm(lib):
    """(sorted instruction addresses, set of return addresses, sorted [(addr, symbol)])"""
    out = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", "-C", lib], capture_output=True, text=True).stdout
    insns, rets, syms = [], set(), []
    prev_call = False
    for line in out.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.*)>:$", line)
        if m:
            syms.append((int(m.group(1), 16), m.group(2)))
            prev_call = False
            continue
        m = re.match(r"^\s+([0-9a-f]+):\s+(\S+)", line)
        if not m:
            continue
        a = int(m.group(1), 16)
        if prev_call:
            rets.add(a)
        insns.append(a)
        prev_call = m.group(2).startswith("call")
    syms.sort()
    return insns, rets, syms


def sym_of(syms, off):
    i = bisect.bisect_right(syms, (off, "￿")) - 1
    return f"{syms[i][1]}+0x{off - syms[i][0]:x}" if i >= 0 else "?"


def main():
    log = open(sys.argv[1]).read()
    libs = sys.argv[2:] or DEFAULT_LIBS
    pc = re.search(r"PC: @\s+0x([0-9a-f]+)", log)
    frames = [int(x, 16) for x in re.findall(r"@\s+0x([0-9a-f]+) ", log.split("stack trace")[-1])]
    fault = int(pc.group(1), 16) if pc else None
    allf = sorted(set(frames + ([fault] if fault else [])))
    print(f"{len(frames)} frames, fault PC {hex(fault) if fault else None}")
    for lib in libs:
        try:
            insns, rets, syms = disasm(lib)
        except Exception as ex:
            print(f"{lib}: {ex}")
            continue
        if not insns:
            continue
        iset = set(insns)
        lo, hi = insns[0], insns[-1]
        best = None
        for f in allf:
            for r in (rets if f != fault else iset):
                if (r & 0xfff) != (f & 0xfff):
                    continue
                base = f - r
                hit = [g for g in allf if (g - base) in (iset if g == fault else rets)]
                if len(hit) >= 2 and (best is None or len(hit) > len(best[1])):
                    best = (base, hit)
        if best:
            base, hit = best
            print(f"\n{lib}: base {hex(base)} explains {len(hit)} frames")
            for g in hit:
                print(f"  {hex(g)}  +0x{g - base:x}  {'FAULT ' if g == fault else ''}{sym_of(syms, g - base)}")
        else:
            print(f"\n{lib}: no consistent base")


if __name__ == "__main__":
    main()
