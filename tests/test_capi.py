"""CPU: the C-ABI library builds, loads and exports exactly the entry points include/vjepa_hip.h
declares (no compute calls: there is no GPU here)."""

import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "vjepa_hip.h")


def declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*int\s+(vj_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_entry_points():
    names = declared()
    assert "vj_gemm_bf16" in names and "vj_attn_fwd" in names and len(names) >= 20


def test_library_exports_every_declared_symbol():
    from vjepa2_amd import _lib

    if not os.path.exists(_lib.LIB_PATH):
        from vjepa2_amd.build import build

        build(verbose=False)
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\sT\s(vj_\w+)", out))
    missing = set(declared()) - exported
    assert not missing, f"declared but not exported: {missing}"
    undeclared = exported - set(declared())
    assert not undeclared, f"exported but not declared in include/vjepa_hip.h: {undeclared}"
    lib = _lib.load()
    for n in declared():
        getattr(lib, n)
    assert set(_lib.SIGNATURES) == set(declared()), "ctypes signatures out of sync with the header"


def test_header_enums_match_host_constants():
    """The epilogue enum of include/vjepa_hip.h carries the same values as vjepa2_amd/ops.py's EPI_*."""
    from vjepa2_amd import ops

    src = open(HEADER).read()
    enum = dict((k, int(v)) for k, v in re.findall(r"VJ_(EPI_\w+)\s*=\s*(\d+)", src))
    host = {k: getattr(ops, k) for k in dir(ops) if re.fullmatch(r"EPI_[A-Z0-9_]+", k) and isinstance(getattr(ops, k), int)}
    assert enum == host, (enum, host)
    assert ops.EPI_NAMES[ops.EPI_BF16_RESID] == "EPI_BF16_RESID"


def test_library_metadata_and_errors():
    from vjepa2_amd import _lib

    lib = _lib.load()
    assert lib.vj_version() == 1
    # argument validation happens before any device work -> usable without a GPU
    rc = lib.vj_gemm_bf16(16, 16, 12, None, 16, 1, None, 16, 1, 0, None, None, 0, None, 16, None, 0, None)
    assert rc != 0 and "null operand" in _lib.last_error()
    for internal in (5, 6, 8):  # RoPE / split-K partial (+ row sums) epilogues are internal: rejected at the C ABI
        rc = lib.vj_gemm_bf16(16, 16, 16, None, 16, 1, None, 16, 1, internal, None, None, 0, None, 16, None, 0, None)
        assert rc != 0 and "not a public epilogue" in _lib.last_error()
    # the fused weight + bias gradient validates before any launch
    rc = lib.vj_gemm_bf16_wgrad(64, 64, 64, None, 64, None, 64, None, 64, 0, None, 0, 1, None, 0, None)
    assert rc != 0 and "null dw" in _lib.last_error()
    rc = lib.vj_attn_fwd(10, 2, 48, None, 288, 0, 96, 192, None, 96, None, 0.1, 1, _lib.int_array([1]),
                         _lib.int_array([10]), None)
    assert rc != 0 and "head_dim" in _lib.last_error()


def test_single_hip_runtime_in_process():
    """Our library must bind to the HIP runtime torch loaded (one runtime per process)."""
    import torch  # noqa: F401

    from vjepa2_amd import _lib

    _lib.load()
    maps = open("/proc/self/maps").read()
    libs = {line.split()[-1] for line in maps.splitlines() if "libamdhip64" in line}
    assert len(libs) == 1, libs


def _kernel_metadata():
    """name -> AMDGPU kernel metadata of every gfx950 kernel in libvjepa_hip.so: the .hip_fatbin
    section holds one clang offload bundle per source; each bundle's gfx950 entry is a code object
    whose NT_AMDGPU_METADATA note llvm-readelf prints as YAML."""
    import struct
    import tempfile

    import pytest
    import yaml

    from vjepa2_amd import _lib

    llvm = "/opt/rocm/lib/llvm/bin"
    if not os.path.exists(os.path.join(llvm, "llvm-readelf")) or not os.path.exists(_lib.LIB_PATH):
        pytest.skip("llvm tools or the library are missing")
    meta = {}
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fatbin")
        subprocess.run([os.path.join(llvm, "llvm-objcopy"), "--dump-section", f".hip_fatbin={fb}", _lib.LIB_PATH,
                        os.path.join(td, "so")], check=True, capture_output=True)
        data = open(fb, "rb").read()
        magic = b"__CLANG_OFFLOAD_BUNDLE__"
        for s in [m.start() for m in re.finditer(re.escape(magic), data)]:
            n = struct.unpack_from("<Q", data, s + 24)[0]
            off = s + 32
            for _ in range(n):
                o, sz, tl = struct.unpack_from("<QQQ", data, off)
                trip = data[off + 24:off + 24 + tl].decode()
                off += 24 + tl
                if "gfx950" not in trip:
                    continue
                elf = os.path.join(td, "co.elf")
                with open(elf, "wb") as f:
                    f.write(data[s + o:s + o + sz])
                out = subprocess.run([os.path.join(llvm, "llvm-readelf"), "--notes", elf], capture_output=True,
                                     text=True, check=True).stdout
                doc = out[out.index("---"):out.rindex("...")]
                for k in yaml.safe_load(doc)["amdhsa.kernels"]:
                    meta[k[".name"]] = k
    return meta


# Scratch the compiler gives kernels that spill a few registers today (measured; documented in DESIGN:
# the dQ sweep reloads one dword per key tile at 3 workgroups per CU, three with attention dropout; the
# one-tile 8-wave GEMM runs at 256 VGPRs): a guard against growth, the rest must stay at zero.
KNOWN_SCRATCH = {r"k_attn_bwd_dqILi64ELi1ELb0E": 8, r"k_attn_bwd_dqILi64ELi1ELb1E": 12, r"k_gemm256ILb[01]ELb1ELi\d+ELi256ELb0ELi8ELi256ELi0E": 20}


def test_hot_kernels_register_budgets():
    """Occupancy the measured kernels rely on, checked from the code objects: the hd-64
    attention forward runs 3 waves per SIMD only at <= 168 VGPRs (FWD_OCC=2 lets the compiler go to
    256, so a later edit or compiler could silently fall to 2); no GEMM or attention kernel spills
    beyond KNOWN_SCRATCH."""
    meta = _kernel_metadata()
    fwd = [k for n, k in meta.items() if "k_attn_fwdILi64ELb0E" in n]  # Lb0E: without attention dropout
    assert fwd, sorted(meta)[:10]
    for k in fwd:
        assert k[".vgpr_count"] + k.get(".agpr_count", 0) <= 168, (k[".name"], k[".vgpr_count"])
    hot = [k for n, k in meta.items() if re.search(r"k_gemm256|k_attn_(fwd|bwd)", n)]
    assert len(hot) >= 40
    for k in hot:
        cap = max([b for pat, b in KNOWN_SCRATCH.items() if re.search(pat, k[".name"])], default=0)
        assert k[".private_segment_fixed_size"] <= cap, (k[".name"], k[".private_segment_fixed_size"], cap)
