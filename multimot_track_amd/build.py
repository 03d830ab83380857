"""Build libmmt.so in-tree with hipcc for gfx950 (no JIT cache; the .so travels with the repo
snapshot to the GPU box).  Flags: -ffp-contract=off (no FMA contraction: bit-exact fp32 with the
CPU oracle) and correctly rounded fp32 division/sqrt."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libmmt.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
         "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt",
         "-Wall", "-Wno-unused-function", "-Wno-unused-variable",
         "-Xarch_host", "-mpopcnt"]  # host: the popcount instruction (map-point descriptors)
FLAGS += os.environ.get("MMT_EXTRA_FLAGS", "").split()  # e.g. -DMMT_LM_PROFILE (tools/)


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC)
                  if f.endswith(".hip") or f.endswith(".cpp"))


def needs_build():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = sources() + [os.path.join(CSRC, f) for f in os.listdir(CSRC)
                        if f.endswith((".h", ".inc"))]
    deps.append(os.path.join(HERE, "..", "include", "mmt.h"))
    return any(os.path.getmtime(d) > t for d in deps)


CLI = os.path.join(HERE, "cli")
IO_LIB = os.path.join(HERE, "libmmt_io.so")
CLI_BIN = os.path.join(HERE, "rgbd_mmt")
CXX = os.environ.get("CXX", "g++")


def build_cli(force=False, verbose=True):
    """Host-only pieces above the C-ABI: libmmt_io.so (sequence decoding) and the rgbd_mmt
    drop-in executable (links libmmt.so through an $ORIGIN rpath)."""
    srcs = [os.path.join(CLI, f) for f in ("mmt_io.cpp", "mmt_io.h", "mmt_viz.h", "rgbd_mmt.cpp")]
    newest = max(os.path.getmtime(s) for s in srcs + [OUT])
    cmds = []
    if force or not os.path.exists(IO_LIB) or os.path.getmtime(IO_LIB) < newest:
        cmds.append([CXX, "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall",
                     os.path.join(CLI, "mmt_io.cpp"), "-lz", "-o", IO_LIB])
    if force or not os.path.exists(CLI_BIN) or os.path.getmtime(CLI_BIN) < newest:
        cmds.append([CXX, "-O2", "-std=c++17", "-Wall", os.path.join(CLI, "rgbd_mmt.cpp"),
                     os.path.join(CLI, "mmt_io.cpp"), "-L" + HERE, "-l:libmmt.so", "-lz",
                     "-Wl,-rpath,$ORIGIN", "-o", CLI_BIN])
    for c in cmds:
        if verbose:
            print(" ".join(c), flush=True)
        subprocess.check_call(c)


def build(force=False, verbose=True):
    if not force and not needs_build():
        build_cli(force, verbose)
        return OUT
    objs = []
    procs = []
    os.makedirs(os.path.join(HERE, "build"), exist_ok=True)
    for src in sources():
        obj = os.path.join(HERE, "build", os.path.basename(src) + ".o")
        cmd = [HIPCC] + [f for f in FLAGS if f != "-shared"] + ["-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append(subprocess.Popen(cmd))
        objs.append(obj)
    for p in procs:
        if p.wait() != 0:
            raise RuntimeError("hipcc failed")
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", OUT] + objs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    build_cli(True, verbose)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
