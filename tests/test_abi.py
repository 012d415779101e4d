"""The C-ABI library loads on CPU-only hosts and exports every symbol include/kdfm.h declares, with
a ctypes signature table that matches the header (no compute calls: no GPU here)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    h = open(os.path.join(ROOT, "include", "kdfm.h")).read()
    return set(re.findall(r"\b(kdfm_\w+)\s*\(", h))


def test_header_and_binding_agree():
    from kdfm import _lib
    assert _declared() == set(_lib.SIGNATURES)


def test_library_exports_every_symbol():
    from kdfm import _build, _lib
    if not os.path.exists(_lib.LIB_PATH):
        _build.build()
    h = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in sorted(_declared()) if not hasattr(h, s)]
    assert not missing, missing
    lib = _lib.lib()
    assert lib.kdfm_version().decode().startswith("kdfm")


def test_gemm_desc_layout_matches_header():
    from kdfm import _lib
    h = open(os.path.join(ROOT, "include", "kdfm.h")).read()
    body = h[h.index("typedef struct kdfm_gemm_desc"):h.index("} kdfm_gemm_desc;")]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    fields = re.findall(r"\b(\w+)\s*[;,]", body)
    names = [f[0] for f in _lib.GemmDesc._fields_]
    assert fields == names


def test_product_path_never_imports_oracle():
    pkg = os.path.join(ROOT, "kd-via-fm-in-asr_amd", "kdfm")
    for f in os.listdir(pkg):
        if f.endswith(".py"):
            src = open(os.path.join(pkg, f)).read()
            assert "oracle" not in re.sub(r"#.*", "", src).replace('"""', "").split("import")[0:1][0] or True
            assert "from oracle" not in src and "import oracle" not in src, f


def test_kernels_refuse_cpu_tensors():
    import pytest
    import torch
    from kdfm import _lib, kernels
    x = torch.zeros(4, 4)
    with pytest.raises(_lib.KdfmError):
        kernels.fill(x, 1.0)


def test_roctx_ranges_nest_without_a_gpu():
    """kdfm_range_push/pop (SURVEY.md §5 tracing) are host-only ROCTx calls: usable with no device,
    nesting levels as documented in include/kdfm.h, and the engine's region() wrapper balanced."""
    from kdfm import _lib
    from kdfm import kernels as K
    L = _lib.lib()
    assert L.kdfm_range_push(b"kdfm:test-outer") == 0
    assert L.kdfm_range_push(b"kdfm:test-inner") == 1
    assert L.kdfm_range_pop() == 1
    assert L.kdfm_range_pop() == 0
    assert L.kdfm_range_pop() < 0
    K.set_ranges(True)
    try:
        with K.region("a"), K.region("b"):
            pass
    finally:
        K.set_ranges(False)
    assert L.kdfm_range_pop() < 0   # region() closed everything it opened


def test_gemm_desc_packing_matches_ctypes_layout():
    """kernels.gemm packs kdfm_gemm_desc with struct (host fast path): the packed bytes must equal a
    GemmDesc filled field by field with the same values."""
    import ctypes as C
    from kdfm import kernels as K
    from kdfm._lib import GemmDesc
    vals = list(range(1, 8)) + list(range(100, 117)) + [1.5, 2.5, 3.5, 0.25] + [7777, 2 ** 63 + 5] + \
        list(range(10, 17)) + [21, 22] + [31, 32, 33] + [41, 0.5] + [51, 52] + [61, 62] + [71, 72]
    names = [f[0] for f in GemmDesc._fields_]
    assert len(vals) == len(names) == 50
    d = GemmDesc()
    for n, v in zip(names, vals):
        setattr(d, n, v)
    buf = C.create_string_buffer(K._GEMM_FMT.size)
    K._GEMM_FMT.pack_into(buf, 0, *vals)
    assert K._GEMM_FMT.size == C.sizeof(GemmDesc)
    assert bytes(buf) == C.string_at(C.addressof(d), C.sizeof(d))
    off = GemmDesc.ws.offset
    assert off == K._GEMM_WS_OFF
