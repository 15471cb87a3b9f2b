"""SGPR-spill lanes in a template kernel's ISA (no GPU needed).

For each function of a code object: the VGPRs that hold spilled SGPRs (the
registers of v_writelane / v_readlane) and how many other instructions -- VALU
results, loads -- write them.  With -amdgpu-prealloc-sgpr-spill-vgprs (jit.cc
kOpts) a spill VGPR is written only by v_writelane and the epilogue's reload;
without it the register allocator shares them with ordinary values through
whole-wave copies, the configuration that faulted on the GPU (DESIGN.md
round-6 table, item 1).

    python tools/isa_spill_lanes.py <code object .co> [function name prefix]
"""
import collections
import re
import subprocess
import sys

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def main():
    co = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else ""
    asm = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", co], capture_output=True, text=True).stdout
    fn = None
    lanes = collections.defaultdict(set)
    defs = collections.defaultdict(collections.Counter)
    for ln in asm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.*)>:", ln)
        if m:
            fn = m.group(1)
            continue
        code = ln.strip().split("//")[0].strip()
        if not code or fn is None:
            continue
        op = code.split()[0]
        args = code[len(op):].strip()
        if op in ("v_writelane_b32", "v_readlane_b32"):
            r = re.findall(r"\bv(\d+)\b", args)
            if r:
                lanes[fn].add(int(r[0]))
            continue
        if op.startswith("v_cmp") or op == "v_readfirstlane_b32" or "store" in op:
            continue
        if op.startswith("v_") or "load" in op:
            first = args.split(",")[0].strip()
            m2 = re.match(r"v\[(\d+):(\d+)\]", first)
            regs = range(int(m2.group(1)), int(m2.group(2)) + 1) if m2 else (
                [int(first[1:])] if re.match(r"^v\d+$", first) else [])
            for r in regs:
                defs[fn][r] += 1
    for f in sorted(lanes):
        if not f.startswith(want):
            continue
        other = {r: defs[f][r] for r in sorted(lanes[f])}
        print("%s\n  spill-lane VGPRs %s; other writes of each: %s" % (f, sorted(lanes[f]), other))


if __name__ == "__main__":
    main()
