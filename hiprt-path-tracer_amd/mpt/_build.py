"""Builds libmpt.so (the HIP path tracer + C ABI) in-tree for gfx950.

Plain hipcc invocations, compiled in parallel, relinked only when a source or
header is newer than the library.  Used by ``__graft_entry__.build()`` and by the
test-suite; never invoked implicitly by the product path (``mpt.lib()`` fails
loudly when the library is missing).
"""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
ROOT = PKG_DIR.parent
CSRC = ROOT / "csrc"
INCLUDE = ROOT.parent / "include"
LIB_PATH = PKG_DIR / "libmpt.so"
OBJ_DIR = CSRC / "build"

SOURCES = ["bvh8.cpp", "mpt_kernels.hip", "bake.hip", "mpt_api.cpp", "image.cpp", "jpeg.cpp"]
# mpt_part.hip is compiled once per part (-DMPT_TU_PART=k): the shading and ReSTIR DI kernel
# instantiations, so that they compile in parallel with the rest
PARTS = [1, 2, 3, 4, 5, 6, 7]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
CXXFLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
    "-Wno-unused-result", "-Wno-unused-value", f"-I{INCLUDE}", f"-I{CSRC}",
]


def _deps() -> list[Path]:
    return [CSRC / s for s in SOURCES] + [CSRC / "mpt_part.hip"] + sorted(CSRC.glob("*.h")) + sorted(INCLUDE.glob("*.h"))


def up_to_date() -> bool:
    if not LIB_PATH.exists():
        return False
    t = LIB_PATH.stat().st_mtime
    return all(p.stat().st_mtime <= t for p in _deps())


def build(force: bool = False, verbose: bool = True, defines=(), out: Path | None = None) -> Path:
    """defines/out: development variants (e.g. -DMPT_SHADE_WAVES=2 into another path)."""
    lib_path = Path(out) if out else LIB_PATH
    if not force and not defines and out is None and up_to_date():
        return LIB_PATH
    obj_dir = OBJ_DIR if out is None else lib_path.parent / "obj"
    obj_dir.mkdir(parents=True, exist_ok=True)
    procs = []
    objs = []
    units = [(s, [], Path(s).stem) for s in SOURCES] + [("mpt_part.hip", [f"-DMPT_TU_PART={k}"], f"mpt_part{k}") for k in PARTS]
    for s, extra, stem in units:
        obj = obj_dir / (stem + ".o")
        objs.append(obj)
        cmd = [HIPCC, *CXXFLAGS, *defines, *extra, "-c", str(CSRC / s), "-o", str(obj)]
        if verbose:
            print("[mpt build]", " ".join(cmd), file=sys.stderr)
        procs.append((stem, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    errors = []
    for s, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            errors.append(f"{s}:\n{out.decode(errors='replace')}")
    if errors:
        raise RuntimeError("libmpt build failed:\n" + "\n".join(errors))
    tmp = lib_path.with_suffix(".so.tmp")
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs)]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    if r.returncode != 0:
        raise RuntimeError("libmpt link failed:\n" + r.stdout.decode(errors="replace"))
    os.replace(tmp, lib_path)
    return lib_path


HOST_DIR = ROOT / "host"
HOST_TEST = HOST_DIR / "gpurenderer_parity"
HOST_SOURCES = [HOST_DIR / "gpu_renderer.cpp", ROOT.parent / "tests" / "cpp" / "gpurenderer_parity.cpp"]


def build_host_test(verbose: bool = True) -> Path:
    """The C++ GPURenderer mirror (host/) linked with libmpt into the test driver of
    tests/test_host_cpp.py (plain g++: the host side is ordinary C++ over the C ABI)."""
    lib = build(verbose=verbose)
    deps = HOST_SOURCES + sorted(HOST_DIR.glob("*.h")) + [lib]
    if HOST_TEST.exists() and all(p.stat().st_mtime <= HOST_TEST.stat().st_mtime for p in deps):
        return HOST_TEST
    # the driver also calls the HIP runtime API itself (hipMalloc'd display buffers)
    cmd = ["g++", "-O2", "-std=c++17", "-D__HIP_PLATFORM_AMD__", f"-I{INCLUDE}", f"-I{HOST_DIR}", "-I/opt/rocm/include",
           *map(str, HOST_SOURCES), f"-L{PKG_DIR}", "-lmpt", "-L/opt/rocm/lib", "-lamdhip64",
           "-Wl,-rpath,$ORIGIN/../mpt", "-Wl,-rpath,/opt/rocm/lib",
           "-Wl,-rpath-link,/opt/rocm/lib", "-o", str(HOST_TEST)]
    if verbose:
        print("[mpt build]", " ".join(cmd), file=sys.stderr)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    if r.returncode != 0:
        raise RuntimeError("host test build failed:\n" + r.stdout.decode(errors="replace"))
    return HOST_TEST


if __name__ == "__main__":
    args = sys.argv[1:]
    defs = [a for a in args if a.startswith("-D")]
    outs = [a[len("--out="):] for a in args if a.startswith("--out=")]
    print(build(force="--force" in args, defines=defs, out=Path(outs[0]) if outs else None))
