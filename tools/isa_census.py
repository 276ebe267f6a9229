#!/usr/bin/env python3
"""ISA instruction census of one kernel's loops.

    python tools/isa_census.py CODE_OBJECT_DISASSEMBLY.s KERNEL_SUBSTRING

The disassembly is `llvm-objdump -d --no-show-raw-insn` of the gfx950 code
object (tools/isa_census.py --extract OBJ writes it from a build object's
.hip_fatbin).  Every backward branch closes a loop [target, branch]; the census
lists each loop's static instruction mix by class: the 64-bit / 32-bit integer
multiplies (v_mad_u64_u32 and v_mul_{lo,hi}_u32 issue at a quarter of the VALU
rate), other VALU, SALU, LDS, vector memory and branches.
"""
import collections
import re
import subprocess
import sys


def extract(obj, out):
    subprocess.check_call(["objcopy", "--dump-section", ".hip_fatbin=/tmp/_fatbin.bin", obj])
    subprocess.check_call(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--unbundle", "--type=o",
                           "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--input=/tmp/_fatbin.bin",
                           "--output=/tmp/_co.o"])
    with open(out, "w") as f:
        subprocess.check_call(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", "--no-show-raw-insn", "/tmp/_co.o"],
                              stdout=f)


def classify(op):
    if op in ("v_mad_u64_u32", "v_mad_i64_i32"):
        return "v_mad_u64_u32 (quarter rate)"
    if op.startswith("v_mul_lo_u32") or op.startswith("v_mul_hi_u32") or op.startswith("v_mul_hi_i32"):
        return "v_mul_lo/hi_u32 (quarter rate)"
    if op.startswith("v_") and ("_f64" in op or op.startswith("v_fma_f64")):
        return "VALU f64"
    if op.startswith("v_readlane") or op.startswith("v_readfirstlane") or op.startswith("v_writelane"):
        return "VALU lane moves"
    if op.startswith("v_"):
        return "VALU other"
    if op.startswith("s_cbranch") or op.startswith("s_branch"):
        return "branch"
    if op.startswith("s_waitcnt") or op.startswith("s_nop") or op.startswith("s_barrier"):
        return "wait/nop/barrier"
    if op.startswith("s_"):
        return "SALU"
    if op.startswith("ds_"):
        return "LDS"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "VMEM"
    return "other"


def main():
    if sys.argv[1] == "--extract":
        return extract(sys.argv[2], sys.argv[3])
    path, name = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^[0-9a-f]+ <.*" + re.escape(name) + r".*>:", l))
    base = int(lines[start].split()[0], 16)
    body = []
    for l in lines[start + 1:]:
        if re.match(r"^[0-9a-f]+ <", l):
            break
        m = re.match(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):", l)
        if m:
            tgt = re.search(r"<[^>]*\+0x([0-9a-f]+)>", l)
            body.append((int(m.group(3), 16), m.group(1), base + int(tgt.group(1), 16) if tgt else None))
    addr_idx = {a: i for i, (a, _, _) in enumerate(body)}
    loops = []
    for i, (a, op, tgt) in enumerate(body):
        if (op.startswith("s_cbranch") or op == "s_branch") and tgt is not None and tgt <= a and tgt in addr_idx:
            loops.append((addr_idx[tgt], i))
    print(f"{name}: {len(body)} instructions, {len(loops)} backward branches")
    for lo, hi in sorted(loops, key=lambda x: -(x[1] - x[0]))[:8]:
        c = collections.Counter(classify(op) for _, op, _ in body[lo:hi + 1])
        print(f"  loop [{lo}, {hi}] ({hi - lo + 1} instructions):")
        for k, v in sorted(c.items(), key=lambda kv: -kv[1]):
            print(f"      {k:34s} {v}")
    c = collections.Counter(classify(op) for _, op, _ in body)
    print("  whole kernel:", dict(sorted(c.items(), key=lambda kv: -kv[1])))


if __name__ == "__main__":
    main()
