#!/usr/bin/env python3
"""Build libmsgpu.so in-tree for gfx950 (hipcc).  Usage: python audio-suite_amd/build.py [--force]"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "msgpu.hip")
OUT = os.path.join(HERE, "msgpu", "libmsgpu.so")
DEPS = [os.path.join(HERE, "csrc", f) for f in os.listdir(os.path.join(HERE, "csrc"))] + \
       [os.path.join(os.path.dirname(HERE), "include", "msgpu.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
         "-Wall", "-Wno-unused-function", "-Wno-unused-value", "-Wno-unused-result"]


def stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(d) > t for d in DEPS)


def build(force: bool = False) -> str:
    if force or stale():
        cmd = [HIPCC, *FLAGS, "-o", OUT + ".tmp", SRC]
        print("[msgpu build]", " ".join(cmd), flush=True)
        subprocess.check_call(cmd)
        os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
