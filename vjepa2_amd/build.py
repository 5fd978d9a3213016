"""Build libvjepa_hip.so (gfx950) in-tree with hipcc.

The library links against the HIP runtime that PyTorch-ROCm already loads (torch/lib/libamdhip64.so,
soname libamdhip64.so.7) so one runtime serves torch's streams and our launches.

    python -m vjepa2_amd.build        # or __graft_entry__.build()
"""

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libvjepa_hip.so")
SOURCES = ["vj_capi.hip", "vj_gemm.hip", "vj_gemm256.hip", "vj_attn.hip", "vj_ops.hip", "vj_f32.hip", "vj_xattn.hip", "vj_variants.hip"]
ARCH = os.environ.get("VJEPA_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -amdgpu-mfma-vgpr-form: MFMA accumulators in arch VGPRs (gfx950 allows it), so the softmax /
# epilogue VALU reads them in place instead of through v_accvgpr_read/write copies.
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-mcode-object-version=5",
          "-mllvm", "-amdgpu-mfma-vgpr-form=1", "-Wno-unused-command-line-argument"]
# Per-source extra flags. Attention: no SLP packing of the softmax f32 math (v_pk_mul_f32 beside
# MFMAs costs issue slots and forces v_mov / v_alignbit shuffles before the bf16 packs).
SRC_FLAGS = {"vj_attn.hip": ["-fno-slp-vectorize"]}


def _torch_libdir():
    try:
        import torch

        return os.path.join(os.path.dirname(torch.__file__), "lib")
    except Exception:  # pragma: no cover
        return None


HEADER = os.path.join(os.path.dirname(HERE), "include", "vjepa_hip.h")


def header_crc():
    """CRC-32 of include/vjepa_hip.h (vj_header_crc in the library; checked by _lib.load)."""
    import zlib

    with open(HEADER, "rb") as f:
        return zlib.crc32(f.read()) & 0xFFFFFFFF


def _needs_build(obj, src, extra=()):
    deps = [src, HEADER, *[os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")], *extra]
    return not os.path.exists(obj) or any(os.path.getmtime(d) > os.path.getmtime(obj) for d in deps)


def build(verbose=True, force=False, variant=None, defines=()):
    """Compile every source for gfx950 and link libvjepa_hip.so. `variant` builds an experimental
    copy (libvjepa_hip_<variant>.so, objects in build/<variant>/) with extra -D `defines`, for
    A/B timing of kernel variants inside one process (tools/bench_kernels.py)."""
    objdir = os.path.join(HERE, "build", variant) if variant else os.path.join(HERE, "build")
    lib = os.path.join(HERE, f"libvjepa_hip_{variant}.so") if variant else LIB
    flags = CFLAGS + [f"-D{d}" for d in defines]
    flags.append(f"-DVJ_HEADER_CRC={header_crc()}u")
    if variant:
        flags.append("-DVJ_VARIANT_BUILD=1")  # unlocks the timing-only VJ_DIAG_* macros (vj_common.h)
        # experiments: extra compiler flags for every source (e.g. VJ_EXTRA_FLAGS=-fno-slp-vectorize)
        flags += os.environ.get("VJ_EXTRA_FLAGS", "").split()
    os.makedirs(objdir, exist_ok=True)
    jobs = []
    csrc = os.environ.get("VJ_CSRC", CSRC) if variant else CSRC  # variant may build another source tree
    for s in SOURCES:
        src = os.path.join(csrc, s)
        obj = os.path.join(objdir, s.replace(".hip", ".o"))
        if force or variant or _needs_build(obj, src):
            jobs.append([HIPCC, *flags, *SRC_FLAGS.get(s, []), "-c", src, "-o", obj])

    def run(cmd):
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        return cmd[-1]

    with ThreadPoolExecutor(max_workers=min(4, max(1, len(jobs)))) as ex:
        for o in ex.map(run, jobs):
            if verbose:
                print(f"[vjepa2_amd.build] compiled {os.path.basename(o)}", file=sys.stderr)
    objs = [os.path.join(objdir, s.replace(".hip", ".o")) for s in SOURCES]
    if force or jobs or not os.path.exists(lib) or any(os.path.getmtime(o) > os.path.getmtime(lib) for o in objs):
        link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib, *objs]
        tl = _torch_libdir()
        if tl:
            link += [f"-L{tl}", f"-Wl,-rpath,{tl}"]
        run(link)
        if verbose:
            print(f"[vjepa2_amd.build] linked {lib}", file=sys.stderr)
    return lib


if __name__ == "__main__":
    args = sys.argv[1:]
    var = None
    if "--variant" in args:
        var = args[args.index("--variant") + 1]
    defs = [a[2:] for a in args if a.startswith("-D")]
    build(force="--force" in args, variant=var, defines=defs)
