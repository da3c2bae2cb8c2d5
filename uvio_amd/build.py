"""Build the in-tree native libraries.

* ``uvio_amd/libuvio_hp.so`` — the product: host orchestration (C++) + gfx950 HIP kernels, C ABI
  declared in ``include/uvio_hp.h``.  Compiled with hipcc --offload-arch=gfx950 only.
* ``uvio_amd/uvio_run_asl`` — the ROS-free serial runner over ASL dataset folders (a C-ABI caller).
* ``oracle/build/liboracle.so`` — the CPU restatement used as the parity checker (test infrastructure).

Usage: ``python -m uvio_amd.build`` (or ``__graft_entry__.build()``).
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "uvio_amd", "csrc")
LIB = os.path.join(ROOT, "uvio_amd", "libuvio_hp.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

SOURCES = [
    "options.cpp",
    "engine_state.cpp",
    "engine_prop.cpp",
    "engine_update.cpp",
    "engine_chain.cpp", "engine_init.cpp",
    "engine_track.cpp",
    "engine_retri.cpp",
    "engine_api.cpp",
    "capi.cpp",
    "shard.cpp",
    "kernels_cov.hip",
    "kernels_ekf.hip",
    "kernels_feat.hip",
    "kernels_chi2.hip",
    "kernels_track.hip",
]


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_product(force=False, verbose=False):
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    hdrs = [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    hdrs.append(os.path.join(ROOT, "include", "uvio_hp.h"))
    if not force and not _newer(LIB, srcs + hdrs):
        return LIB
    objdir = os.path.join(ROOT, "build", "obj")
    os.makedirs(objdir, exist_ok=True)
    objs = []
    procs = []
    for s in srcs:
        o = os.path.join(objdir, os.path.basename(s) + ".o")
        objs.append(o)
        if not force and not _newer(o, [s] + hdrs):
            continue
        cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
               "-Wall", "-Wno-unused-variable", "-Wno-unused-but-set-variable",
               "-I", os.path.join(ROOT, "include"), "-c", s, "-o", o]
        if s.endswith(".hip"):
            cmd[1:1] = ["-x", "hip"]
        if verbose:
            print(" ".join(cmd))
        procs.append((s, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    for s, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            sys.stderr.write(out.decode())
            raise RuntimeError("hipcc failed on %s" % s)
        elif verbose and out:
            sys.stderr.write(out.decode())
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", LIB] + objs + ["-ldl"]
    subprocess.check_call(cmd)
    return LIB


RUNNER = os.path.join(ROOT, "uvio_amd", "uvio_run_asl")


def build_runner(force=False):
    """uvio_amd/uvio_run_asl: the ROS-free serial runner over ASL dataset folders (csrc/run_asl.cpp), a plain
    C++ caller of the C ABI (g++, libuvio_hp.so found next to it, zlib for the PNGs)"""
    src = os.path.join(CSRC, "run_asl.cpp")
    deps = [src, os.path.join(ROOT, "include", "uvio_hp.h"), LIB]
    if not force and not _newer(RUNNER, deps):
        return RUNNER
    cmd = ["g++", "-O2", "-std=c++17", "-Wall", "-I", os.path.join(ROOT, "include"), src, "-o", RUNNER,
           "-L", os.path.dirname(LIB), "-luvio_hp", "-Wl,-rpath,$ORIGIN", "-lz"]
    subprocess.check_call(cmd)
    return RUNNER


def build_oracle():
    odir = os.path.join(ROOT, "oracle")
    subprocess.check_call(["make", "-s", "-C", odir])
    return os.path.join(odir, "build", "liboracle.so")


def build_all(force=False, verbose=False):
    lib = build_product(force=force, verbose=verbose)
    run = build_runner(force=force)
    orc = build_oracle()
    return lib, run, orc


if __name__ == "__main__":
    print(build_all(force="--force" in sys.argv, verbose="-v" in sys.argv))
