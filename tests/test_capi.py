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
    for internal in (5, 6):  # RoPE / split-K partial epilogues are internal: rejected at the C ABI
        rc = lib.vj_gemm_bf16(16, 16, 16, None, 16, 1, None, 16, 1, internal, None, None, 0, None, 16, None, 0, None)
        assert rc != 0 and "not a public epilogue" in _lib.last_error()
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
