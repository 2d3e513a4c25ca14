"""The C-ABI library loads on a GPU-less host and exports exactly what
include/pis_capi.h declares (no compute calls here)."""
import os
import re

from physics_informed_image_segmentation_amd import _hip

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    text = open(os.path.join(ROOT, "include", "pis_capi.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pis_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_bound_symbols():
    assert header_symbols() == sorted(_hip.exported_symbols())


def test_library_loads_and_exports_every_symbol():
    lib = _hip.lib()
    for name in header_symbols():
        assert hasattr(lib, name), name
    assert lib.pis_version() == 1


def test_workspace_queries_run_on_host():
    lib = _hip.lib()
    assert lib.pis_loss_ws(8, 512, 512) > 0
    assert lib.pis_conv3x3_wgrad_ws(8, 512, 512, 64, 64) > 0
    assert lib.pis_convt2x2_wgrad_ws(8, 256, 256, 128, 64) > 0


def test_argument_errors_are_reported_not_thrown():
    lib = _hip.lib()
    rc = lib.pis_conv3x3_fwd(0, 4, 0, 0, 0, 0, 4, 1, 4, 4, 4, 4, 0, 0)
    assert rc == -1
    assert b"pis_conv3x3_fwd" in lib.pis_last_error()


def test_head_loss_fwd_ok_bounds_lds():
    """The fused head + loss forward is refused (the Python side then takes pis_head_fwd +
    pis_loss_fwd) when its staged rows would exceed a workgroup's 160 KB of LDS:
    B = 128 at 1024^2 doubles the bands to 64 rows, (64 + 2) x 1032 x 4 B = 272 KB."""
    lib = _hip.lib()
    assert lib.pis_head_loss_fwd_ok(8, 512, 512, 64) == 1
    assert lib.pis_head_loss_fwd_ok(8, 1024, 1024, 64) == 1
    assert lib.pis_head_loss_fwd_ok(128, 1024, 1024, 64) == 0
    assert lib.pis_head_loss_fwd_ok(1, 16, 1280, 64) == 1
