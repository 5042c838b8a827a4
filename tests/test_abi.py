"""CPU tests of the drop-in boundary: libddq_hip.so loads, exports every
symbol include/ddq_hip.h declares, the ctypes binding covers exactly that
set, and the product path fails loudly without a GPU (no CPU fallback)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ddq_hip.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(?:int|int64_t|double|const char\*)\s+(ddq_\w+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    from ddq import _lib
    if not os.path.exists(_lib.LIB_PATH):
        import subprocess
        subprocess.run(["make", "-C", os.path.join(ROOT, "distributed-deep-q_amd")], check=True)
    return _lib.load()


def test_header_declares_expected_surface():
    fns = header_functions()
    assert len(fns) >= 40
    for must in ("ddq_create", "ddq_replay_sample", "ddq_forward_backward", "ddq_apply",
                 "ddq_allreduce_grads", "ddq_step_graph_async", "ddq_select_action"):
        assert must in fns


def test_library_exports_every_header_symbol(lib):
    missing = [f for f in header_functions() if not hasattr(lib, f)]
    assert not missing, missing


def test_ctypes_binding_matches_header():
    from ddq import _lib
    assert sorted(_lib.EXPORTED) == header_functions()


def test_struct_layouts_match_header():
    from ddq import _lib
    # offsets implied by the C declarations in include/ddq_hip.h (x86-64 SysV)
    assert ctypes.sizeof(_lib.NetDesc) == 20
    assert ctypes.sizeof(_lib.BlobDesc) == 16 + 4 + 16 + 4 + 8 + 8   # incl. padding
    assert _lib.BlobDesc.offset.offset == 40
    assert ctypes.sizeof(_lib.UpdateCfg) == 24
    assert ctypes.sizeof(_lib.StepCfg) == 24 + 4 + 4 + 8 + 4 + 4
    assert _lib.StepCfg.seed.offset == 32 and _lib.StepCfg.overlap.offset == 40


def test_abi_version(lib):
    assert lib.ddq_abi_version() == 6


@pytest.mark.parametrize("batch,frame,ok", [(1024, 256, True), (1024, 512, False),
                                            (128, 1016, True), (131, 1016, False),
                                            (1, 1024, False)])
def test_create_rejects_sizes_past_32bit_offsets(lib, batch, frame, ok):
    """ddq_create refuses shapes whose tensors exceed the kernels' 32-bit
    buffer offsets (16 B S^2 and 2^11 S^2 bytes < 2^31), before it looks for
    a device: those sizes fail with DDQ_EINVAL on any host."""
    from ddq import _lib
    desc = _lib.NetDesc(batch, frame, 4, 4, 0.85)
    ctx = ctypes.c_void_p()
    rc = lib.ddq_create(ctypes.byref(ctx), 0, ctypes.byref(desc))
    if ok:
        assert rc != _lib.DDQ_EINVAL or b"32-bit" not in lib.ddq_last_error(None)
        if rc == 0:
            lib.ddq_destroy(ctx)
    else:
        assert rc == _lib.DDQ_EINVAL
        assert b"32-bit" in lib.ddq_last_error(None)


def test_no_gpu_fails_loudly(lib):
    """Without a device the product path raises; it never computes on the CPU."""
    import ddq
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        pytest.skip("GPU present")
    with pytest.raises(ddq._lib.DDQError) as ei:
        ddq.DeepQNet(batch=4, frame=16)
    assert ei.value.code == ddq._lib.DDQ_EHIP


def test_missing_library_raises(tmp_path):
    from ddq import _lib
    saved = _lib._lib
    try:
        _lib._lib = None
        with pytest.raises(ImportError):
            _lib.load(str(tmp_path / "nope.so"))
    finally:
        _lib._lib = saved


def test_header_constants_match_binding():
    """ddq/_lib.py's copies of the header's #defines (step flags, ABI version)."""
    from ddq import _lib
    txt = open(HEADER).read()
    defs = {k: int(v) for k, v in re.findall(r"#define\s+(DDQ_\w+)\s+(\d+)", txt)}
    assert defs["DDQ_ABI_VERSION"] == _lib.ABI_VERSION
    assert defs["DDQ_STEP_NO_GRAD_STORE"] == _lib.STEP_NO_GRAD_STORE
    assert "DDQ_STEP_REPEAT_CONV2_FWD" not in defs          # ABI 6: removed (refused)
    enums = dict((k, int(v)) for k, v in re.findall(r"(DDQ_FAULT_\w+)\s*=\s*(\d+)", txt))
    assert enums == {"DDQ_FAULT_NONE": _lib.FAULT_NONE,
                     "DDQ_FAULT_MEET_TIMEOUT": _lib.FAULT_MEET_TIMEOUT}
