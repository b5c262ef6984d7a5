"""Builds the in-tree HIP engine library raftd_amd/libraftgpu.so for gfx950 (hipcc), and the
test oracle oracle/build/liboracle.so (gcc). Run: python -m raftd_amd.build"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libraftgpu.so")
RESOURCES = os.path.join(PKG, "kernel_resources.txt")  # per-kernel VGPR / scratch / occupancy of the last build
# (source, extra flags, object): the control kernel is compiled once per replica count and the payload
# kernel once per (wire, multi-job) variant, so the heavy instantiations build in parallel
UNITS = ([("raftgpu_ctl.hip", [f"-DRG_CTL_R={r}"], f"raftgpu_ctl{r}.o") for r in range(8, 0, -1)]
         + [("raftgpu_bulk.hip", [f"-DRG_BULK_W={w}", f"-DRG_BULK_MJ={m}"], f"raftgpu_bulk_w{w}m{m}.o")
            for w in (0, 1) for m in (0, 1)]
         + [(f, [], f.rsplit(".", 1)[0] + ".o") for f in ("raftgpu_kernels.hip", "raftgpu_admin.hip", "raftgpu_wire.hip",
                                                          "raftgpu_apply.hip", "raftgpu_engine.cpp", "raftgpu_rccl.cpp",
                                                          "raftgpu_sdma.cpp")])
SOURCES = sorted({u[0] for u in UNITS})
HEADERS = ["raftgpu_internal.h", "raftgpu_control.h", "raftgpu_dev.h", "raftgpu_wire.h", "raftgpu_sdma.h",
           os.path.join("..", "..", "include", "raftgpu.h")]
ARCH = os.environ.get("RAFTGPU_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _stale(out: str, deps: list[str]) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def _digest(deps: list[str]) -> str:
    """Content hash of the sources a library was built from (a build that raced an edit shows up as
    a mismatch, which mtimes alone miss)."""
    import hashlib
    h = hashlib.sha256()
    for d in deps:
        with open(d, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def build_engine(force: bool = False, verbose: bool = False, out: str | None = None, extra: tuple = ()) -> str:
    """Compile and link libraftgpu.so. out / extra: an experimental variant (ablation builds,
    scripts/build_variant.sh) with extra compiler flags, linked into another file; the product build
    is out=None, extra=()."""
    import tempfile
    from concurrent.futures import ThreadPoolExecutor
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    variant = out is not None
    lib = os.path.abspath(out) if variant else LIB
    stamp = LIB + ".sha256"
    digest = _digest(deps)  # taken before compiling: an edit during the build leaves the stamp stale
    if (not variant and not force and not _stale(LIB, deps) and os.path.exists(RESOURCES) and os.path.exists(stamp)
            and open(stamp).read().strip() == digest):
        return LIB
    odir = tempfile.mkdtemp(prefix="raftgpu_obj_")

    def compile_one(unit):
        src, flags, oname = unit
        obj = os.path.join(odir, oname)
        if src.endswith(".hip"):
            lang = [f"--offload-arch={ARCH}", "-x", "hip"]
        else:  # host-only runtime (no device pass: TickParams' device-side address spaces stay out of it)
            lang = ["-x", "c++", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"]
        cmd = ([HIPCC] + lang + ["-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function"] + list(flags)
               + list(extra) + ["-c", os.path.join(CSRC, src), "-o", obj])
        if src.endswith(".hip"):
            cmd.append("-Rpass-analysis=kernel-resource-usage")
        if verbose:
            print(" ".join(cmd))
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"{src} {' '.join(flags)}: hipcc failed\n{r.stderr[-8000:]}")
        rep = [ln.split("remark: ", 1)[1].split(" [-Rpass")[0].strip()
               for ln in r.stderr.splitlines() if "kernel-resource-usage" in ln and "remark: " in ln]
        other = [ln for ln in r.stderr.splitlines() if "warning:" in ln or "error:" in ln]
        return obj, rep, other

    # the units compile in parallel, the slowest (most replicas) first
    jobs = max(1, min(len(UNITS), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1))))
    with ThreadPoolExecutor(jobs) as ex:
        results = list(ex.map(compile_one, UNITS))
    objs, report = [], []
    for obj, rep, other in results:
        if other:
            print("\n".join(other), file=sys.stderr)
        objs.append(obj)
        report += rep
    if not variant:
        with open(RESOURCES, "w") as f:
            f.write("\n".join(report) + "\n")
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib] + objs + ["-ldl"]
    subprocess.run(cmd, check=True)
    for o in objs:
        os.remove(o)
    os.rmdir(odir)
    if not variant:
        with open(stamp, "w") as f:
            f.write(digest + "\n")
    return lib


def build_oracle() -> str:
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    return os.path.join(ROOT, "oracle", "build", "liboracle.so")


def build_abi_harness() -> str:
    """gcc the plain-C ABI harness tests/native/abi_c.c (the call sequence a cgo shim makes) against
    the in-tree libraftgpu.so: tests/native/abi_c.bin (test infrastructure, run by tests/test_abi.py)."""
    src = os.path.join(ROOT, "tests", "native", "abi_c.c")
    out = os.path.join(ROOT, "tests", "native", "abi_c.bin")
    lib = build_engine()
    deps = [src, lib, os.path.join(ROOT, "include", "raftgpu.h")]
    if not _stale(out, deps):
        return out
    subprocess.run(["gcc", "-O2", "-std=c11", "-Wall", "-Wextra", "-Werror", src, "-I", os.path.join(ROOT, "include"),
                    "-L", PKG, "-lraftgpu", "-lz", "-Wl,-rpath,$ORIGIN/../../raftd_amd", "-Wl,-rpath,/opt/rocm/lib",
                    "-o", out], check=True)
    return out


def main():
    if "--variant" in sys.argv:  # python -m raftd_amd.build --variant OUT.so -DFLAG ... (ablation builds)
        i = sys.argv.index("--variant")
        print(build_engine(out=sys.argv[i + 1], extra=tuple(sys.argv[i + 2:])))
        return
    force = "--force" in sys.argv
    print(build_engine(force=force, verbose=True))
    print(build_oracle())
    print(build_abi_harness())


if __name__ == "__main__":
    main()


def kernel_resources() -> dict:
    """{kernel name: {field: value}} from the last build's resource-usage remarks."""
    build_engine()
    out, cur = {}, None
    for ln in open(RESOURCES):
        k, _, v = ln.strip().partition(": ")
        if k == "Function Name":
            cur = out.setdefault(v, {})
        elif cur is not None:
            cur[k] = v
    return out
