"""The C-ABI library loads here (no GPU) and exports every symbol include/impala_hip.h
declares; host-only entry points and argument validation work without a device."""
import ctypes as C
import os
import re
import subprocess

import pytest

from impala_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "impala_hip.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(impala_\w+)\s*\(", src)))


def test_header_declares_what_the_binding_expects():
    assert _declared() == sorted(_lib.EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = _lib.lib()
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\b(impala_\w+)\b", out))
    for name in _declared():
        assert name in exported, name
        assert hasattr(lib, name)


def test_host_only_entry_points():
    lib = _lib.lib()
    assert lib.impala_abi_version() == _lib.ABI_VERSION == 3
    assert _lib.param_count(15) == 344496
    assert _lib.param_count(6) == 344496 - 9 * 257
    cfg = _lib.default_config()
    assert (cfg.batch_size, cfg.rollout_length, cfg.num_actions) == (8, 20, 15)
    assert abs(cfg.lr - 1e-4) < 1e-9 and abs(cfg.adam_eps - 1e-5) < 1e-12
    assert abs(cfg.max_grad_norm - 0.5) < 1e-9 and abs(cfg.entropy_coeff - 0.01) < 1e-9
    assert cfg.vtrace_grad_mode == _lib.VTRACE_GRAD_MODES["sg_advantage"] == 0
    names = [lib.impala_kernel_name(i).decode() for i in range(lib.impala_kernel_count())]
    assert "conv2_dgrad_conv1_wgrad" in names and "adam" in names and len(names) == len(set(names))


@pytest.mark.parametrize("field,value", [("batch_size", 0), ("rollout_length", 1),
                                         ("rollout_length", 65), ("num_actions", 16),
                                         ("num_actions", 0), ("dtype", 7), ("world_size", 0),
                                         ("algo", 5), ("ppo_clip", 1.5),
                                         ("vtrace_grad_mode", 3), ("vtrace_grad_mode", -1)])
def test_create_rejects_bad_config_without_touching_the_device(field, value):
    lib = _lib.lib()
    cfg = _lib.default_config()
    setattr(cfg, field, value)
    h = C.c_void_p()
    st = lib.impala_create(C.byref(cfg), 0, C.byref(h))
    assert st in (1001, 1003)
    assert not h.value
    assert lib.impala_last_error().decode()


def test_kernel_entry_points_validate_before_launch():
    lib = _lib.lib()
    assert lib.impala_vtrace(None, None, None, None, None, 4, 0, 1.0, 1.0, 1.0, None, None,
                             None, None) == 1001
    assert lib.impala_vtrace(None, None, None, None, None, 4, 65, 1.0, 1.0, 1.0, None, None,
                             None, None) == 1001
    assert lib.impala_loss_head(*([None] * 6), 2, 1, 15, 0.01, 1.0, 1.0, 1.0, 1,
                                *([None] * 8)) == 1001
    assert lib.impala_loss_head(*([None] * 6), 2, 20, 15, 0.01, 1.0, 1.0, 1.0, 9,
                                *([None] * 8)) == 1001
    assert lib.impala_train_step(None, None, None) == 1001
    assert lib.impala_forward(None, None, 1, None, None, None) == 1001
    assert lib.impala_gather_rows(None, None, None, 0, None, 0, None) == 1001
    # host staging ring: a null handle is refused before any HIP call
    assert lib.impala_stage_init(None, 2) == 1001
    assert lib.impala_stage(None, None, 0) == 1001
    assert lib.impala_stage_wait(None, 0) == 1001
    assert lib.impala_slot_batch(None, 0, None, None) == 1001
    assert lib.impala_slot_release(None, 0, None) == 1001
    assert lib.impala_act(None, None, 1, None, 0, 0, 0, None, None, None, None) == 1001
    # device step clock: a null handle is refused before any HIP call
    assert lib.impala_step_clock(None, None, 3) == 1001
    assert lib.impala_step_clock_end(None, None, None) == 1001


def test_headers_compile_as_c99(tmp_path):
    """include/*.h are the boundary a C (or cgo / FFI) binding includes: they must be plain C99,
    with no C++ in the declarations."""
    import os
    import shutil
    import subprocess
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    src = tmp_path / "hdr.c"
    src.write_text('#include "impala_hip.h"\n#include "sac_hip.h"\n'
                   "int main(void) { return IMPALA_NUM_METRICS == 9 ? 0 : 1; }\n")
    r = subprocess.run([cc, "-std=c99", "-Wall", "-Werror", "-I", inc, "-c", str(src), "-o",
                        str(tmp_path / "hdr.o")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
