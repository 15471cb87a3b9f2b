"""Histogram of host-trap PC samples (rocprofv3 --pc-sampling ... --output-format csv,
tools/gpu_pcsample.sh) over one code object, annotated with its disassembly.

usage: python tools/pc_hist.py <pc_sampling csv> <code object .co> [top N]
Prints the hottest instructions (offset, samples, share, instruction, the
function they belong to) and the share of samples per function and per
instruction class (global/scratch/flat/ds memory, waitcnt, branch, valu,
salu)."""
import collections
import csv
import re
import subprocess
import sys

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def disasm(co):
    out = subprocess.run([OBJDUMP, "-d", "--arch-name=amdgcn", "--mcpu=gfx950", co], capture_output=True,
                         text=True).stdout
    ins, func = {}, {}
    cur = "?"
    for line in out.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.+)>:", line)
        if m:
            cur = m.group(2)
            continue
        m = re.match(r"^\s+(\S.*?)\s*//\s*([0-9A-F]+):", line)
        if m:
            a = int(m.group(2), 16)
            ins[a] = m.group(1)
            func[a] = cur
    return ins, func


def klass(text):
    op = text.split()[0] if text else "?"
    for p in ("global_load", "global_store", "global_atomic", "scratch_", "flat_", "buffer_", "ds_", "s_waitcnt",
              "s_load", "s_cbranch", "s_branch", "v_readlane", "v_writelane", "v_readfirstlane", "s_swappc",
              "s_setpc", "v_", "s_"):
        if op.startswith(p):
            return p
    return op


def main():
    path, co = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 60
    rows = list(csv.DictReader(open(path)))
    if not rows:
        print("no samples")
        return
    cols = list(rows[0].keys())
    off_col = next((c for c in cols if "offset" in c.lower()), None)
    id_col = next((c for c in cols if "code_object_id" in c.lower().replace(" ", "_")), None)
    print("columns:", cols)
    by_obj = collections.Counter(r.get(id_col, "?") for r in rows)
    print("samples per code object:", by_obj.most_common(8))
    obj = by_obj.most_common(1)[0][0]
    hist = collections.Counter(int(r[off_col], 0) for r in rows if r.get(id_col, "?") == obj)
    total = sum(hist.values())
    ins, func = disasm(co)
    per_func, per_class = collections.Counter(), collections.Counter()
    for a, n in hist.items():
        per_func[func.get(a, "?")] += n
        per_class[klass(ins.get(a, ""))] += n
    print("code object %s: %d samples" % (obj, total))
    print("by function:")
    for f, n in per_func.most_common(15):
        print("  %6.2f%%  %s" % (100.0 * n / total, f[:100]))
    print("by instruction class (the sampled PC is the instruction the wave waits to issue):")
    for k, n in per_class.most_common(20):
        print("  %6.2f%%  %s" % (100.0 * n / total, k))
    print("hottest instructions:")
    for a, n in hist.most_common(top):
        print("  %08x %6d %5.2f%%  %-60s %s" % (a, n, 100.0 * n / total, ins.get(a, "?")[:60], func.get(a, "?")[:40]))


if __name__ == "__main__":
    main()
