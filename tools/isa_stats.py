#!/usr/bin/env python3
"""Per-kernel ISA statistics of libmpasdyn's gfx950 code (LP = 64 instances): vector and
scalar loads, full vmcnt(0) drains, divergent branches, VGPRs, occupancy.  Compiles each
csrc/*.hip to assembly with the library's flags.

usage: python tools/isa_stats.py [file.hip ...]
"""
import glob
import os
import re
import subprocess
import sys

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpas-regent_amd", "csrc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
         "-I" + os.path.join(CSRC, "..", "..", "include"), "-I" + CSRC, "--cuda-device-only", "-S"]


def stats(src):
    out = "/tmp/isa_" + os.path.basename(src) + ".s"
    subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, "-o", out, src], check=True, stderr=subprocess.DEVNULL)
    s = open(out).read()
    meta = dict(re.findall(r"\.name:\s+(\S+)\n(?:(?!\.name:)[\s\S])*?\.vgpr_count:\s+(\d+)", s))
    for m in re.finditer(r"^(_Z\S*ILi64E\S*):\s*(?:;.*)?$", s, re.M):
        name = m.group(1)
        end = s.index(".Lfunc_end", m.end())
        body = s[m.end():end]
        c = lambda p: len(re.findall(p, body))
        short = re.sub(r"^_ZN4mpas\d+", "", name).split("ILi")[0] + (name.split("ILi64E")[1][:int(os.environ.get("ISA_FULL", "12")) if os.environ.get("ISA_FULL", "").isdigit() else 12] if os.environ.get("ISA_FULL") else "")
        v = int(meta.get(name, 0))
        print("%-14s vgpr %3d vload %3d sload %3d vstore %3d vmcnt0 %3d execz %3d valu %4d addr64 %3d f64 %4d insts %5d" % (
            short, v, c(r"global_load|buffer_load"), c(r"s_load"), c(r"global_store"), c(r"vmcnt\(0\)"),
            c(r"execz"), c(r"\n\s+v_"), c(r"v_lshl_add_u64|v_add_co_u32|v_lshlrev_b64"), c(r"\n\s+v_\w+_f64"),
            body.count("\n")))


if __name__ == "__main__":
    for f in sys.argv[1:] or sorted(glob.glob(os.path.join(CSRC, "*.hip"))):
        stats(f)
