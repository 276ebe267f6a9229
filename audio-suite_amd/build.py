#!/usr/bin/env python3
"""Build libmsgpu.so in-tree for gfx950 with hipcc (translation units in parallel).

    python audio-suite_amd/build.py [--force] [--stamps]

--stamps builds msgpu/libmsgpu_stamps.so with per-phase clock stamps in the
spectral kernel (-DMSG_STAMPS, read by tools/spec_stamps.py); load it with
MSGPU_LIB=.../libmsgpu_stamps.so.  Never the product library.

--exp builds msgpu/libmsgpu_exp.so for tuning experiments with the extra defines
in MSGPU_EXP_DEFS (e.g. MSGPU_EXP_DEFS="-DMSG_ST_TILE=2048"); load it with
MSGPU_LIB=.../libmsgpu_exp.so.  Never the product library.

Objects are cached per variant and rebuilt when a source or local header is
newer, or when the variant's defines differ from those recorded in the object
directory's defs stamp (so changing MSGPU_EXP_DEFS always recompiles).

--exp-tu NAME[,NAME..] [--out FILE] is the fast form of --exp for one-kernel
experiments: only the named translation units are compiled (with
MSGPU_EXP_DEFS, into build_exp_tu/, always from scratch) and linked with the
product build's objects for the rest; the library goes to msgpu/FILE
(default libmsgpu_exp.so).  Never the product library.
"""
import concurrent.futures as cf
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "build")
OUT = os.path.join(HERE, "msgpu", "libmsgpu.so")
TUS = ["msgpu.hip", "k_spectral.hip", "k_spectral_ct.hip", "k_spec3.hip", "k_fir.hip", "k_grain64.hip", "k_grain64_lds.hip",
       "k_grain64_glb.hip", "k_stereo_odd.hip", "k_fir64.hip", "k_stereo.hip", "k_digest.hip"]
HEADERS = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")] + \
          [os.path.join(os.path.dirname(HERE), "include", "msgpu.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
         "-Wall", "-Wno-unused-function", "-Wno-unused-value", "-Wno-unused-result"]
# host-side code generation of the TU that holds the render's host planning and
# records (msgpu.hip): SSE4.1 turns rint / nearbyint into one roundsd instead of
# a libm call (plan_sizes 0.63 -> 0.43 us, plan_events 2.9 -> 2.2 us per H48
# preset on this container); no FMA, so host float results keep their bits
TU_HOST_FLAGS = {"msgpu.hip": ["-Xarch_host", "-msse4.1"]}


_INC = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)


def _deps(path, seen=None):
    """Local headers a source includes, transitively (quoted includes only)."""
    seen = set() if seen is None else seen
    with open(path) as f:
        text = f.read()
    for inc in _INC.findall(text):
        h = os.path.normpath(os.path.join(os.path.dirname(path), inc))
        if os.path.exists(h) and h not in seen:
            seen.add(h)
            _deps(h, seen)
    return seen


def _newest_dep(src):
    return max([os.path.getmtime(src)] + [os.path.getmtime(h) for h in _deps(src)])


VARIANTS = {"": ([], "build", "libmsgpu.so"), "stamps": (["-DMSG_STAMPS"], "build_stamps", "libmsgpu_stamps.so"),
            # tuning experiments: python build.py --exp with MSGPU_EXP_DEFS="-DNAME=V ..."
            "exp": (os.environ.get("MSGPU_EXP_DEFS", "").split(), "build_exp", "libmsgpu_exp.so")}


def _defs_stamp(variant):
    """Drop the variant's cached objects when its defines changed since they were
    built (the stamp file records the defines and flags of the objects)."""
    defs, objdir, _ = VARIANTS[variant]
    d = os.path.join(HERE, objdir)
    stamp = os.path.join(d, "defs.stamp")
    want = " ".join(FLAGS + defs + [f"{k}:{' '.join(v)}" for k, v in sorted(TU_HOST_FLAGS.items())])
    try:
        with open(stamp) as f:
            have = f.read()
    except OSError:
        have = None
    if have != want:
        for tu in TUS:
            o = os.path.join(d, tu.replace(".hip", ".o"))
            if os.path.exists(o):
                os.remove(o)
        with open(stamp, "w") as f:
            f.write(want)


def _compile(tu, variant=""):
    defs, objdir, _ = VARIANTS[variant]
    src = os.path.join(CSRC, tu)
    obj = os.path.join(HERE, objdir, tu.replace(".hip", ".o"))
    if os.path.exists(obj) and os.path.getmtime(obj) >= _newest_dep(src):
        return obj
    cmd = [HIPCC, *FLAGS, *TU_HOST_FLAGS.get(tu, []), *defs, "-c", "-o", obj + ".tmp", src]
    print("[msgpu build]", " ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(obj + ".tmp", obj)
    return obj


def build_pack() -> str:
    """The native params-dict packer msgpu/_mspack (csrc/mspack.c, CPython C API,
    host only): rebuilt when the source or include/msgpu.h is newer."""
    import sysconfig
    src = os.path.join(CSRC, "mspack.c")
    out = os.path.join(HERE, "msgpu", "_mspack" + sysconfig.get_config_var("EXT_SUFFIX"))
    newest = max(os.path.getmtime(src), os.path.getmtime(os.path.join(os.path.dirname(HERE), "include", "msgpu.h")))
    if not os.path.exists(out) or os.path.getmtime(out) < newest:
        cmd = [os.environ.get("CC", "gcc"), "-O2", "-shared", "-fPIC", "-Wall", "-Werror",
               "-I" + sysconfig.get_paths()["include"], "-o", out + ".tmp", src]
        print("[msgpu build]", " ".join(cmd), flush=True)
        subprocess.check_call(cmd)
        os.replace(out + ".tmp", out)
    return out


def build(force: bool = False, variant: str = "") -> str:
    _, objdir, libname = VARIANTS[variant]
    out = os.path.join(HERE, "msgpu", libname)
    os.makedirs(os.path.join(HERE, objdir), exist_ok=True)
    if force:
        for tu in TUS:
            o = os.path.join(HERE, objdir, tu.replace(".hip", ".o"))
            if os.path.exists(o):
                os.remove(o)
    _defs_stamp(variant)
    build_pack()
    with cf.ThreadPoolExecutor(max_workers=len(TUS)) as ex:
        objs = list(ex.map(lambda tu: _compile(tu, variant), TUS))
    OUT = out
    if not os.path.exists(OUT) or any(os.path.getmtime(o) > os.path.getmtime(OUT) for o in objs):
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", OUT + ".tmp", *objs]
        print("[msgpu build]", " ".join(cmd), flush=True)
        subprocess.check_call(cmd)
        os.replace(OUT + ".tmp", OUT)
    return OUT


def build_exp_tu(tus, out_name="libmsgpu_exp.so") -> str:
    """Experiment library: `tus` compiled with MSGPU_EXP_DEFS, the rest from the product build.

    The product objects are used as they are (built only when one is missing):
    rebuilding them here would compile an experiment's modified sources into the
    product library too, and an A/B against it would compare a variant with
    itself."""
    if not all(os.path.exists(os.path.join(OBJ, tu.replace(".hip", ".o"))) for tu in TUS):
        build()
    defs = os.environ.get("MSGPU_EXP_DEFS", "").split()
    objdir = os.path.join(HERE, "build_exp_tu")
    os.makedirs(objdir, exist_ok=True)
    objs = []
    for tu in TUS:
        if tu in tus:
            o = os.path.join(objdir, tu.replace(".hip", ".o"))
            cmd = [HIPCC, *FLAGS, *TU_HOST_FLAGS.get(tu, []), *defs, "-c", "-o", o, os.path.join(CSRC, tu)]
            print("[msgpu build]", " ".join(cmd), flush=True)
            subprocess.check_call(cmd)
        else:
            o = os.path.join(HERE, "build", tu.replace(".hip", ".o"))
        objs.append(o)
    out = os.path.join(HERE, "msgpu", out_name)
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out, *objs])
    return out


if __name__ == "__main__":
    if "--exp-tu" in sys.argv:
        tus = sys.argv[sys.argv.index("--exp-tu") + 1].split(",")
        name = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else "libmsgpu_exp.so"
        print(build_exp_tu(tus, name))
        sys.exit(0)
    var = "stamps" if "--stamps" in sys.argv else ("exp" if "--exp" in sys.argv else "")
    print(build(force="--force" in sys.argv, variant=var))
