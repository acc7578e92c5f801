"""The C-ABI library loads and exports every entry point include/vosdet.h
declares (no compute: this runs on the CPU host too)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "vosdet.h")


def declared():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(vd_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_entry_points():
    names = declared()
    for must in ["vd_roi_align_forward", "vd_roi_align_backward", "vd_roi_align_fpn_forward",
                 "vd_nms", "vd_generate_proposals", "vd_collect_distribute",
                 "vd_box_detections", "vd_roi_pool_forward", "vd_roi_crop_forward",
                 "vd_roi_align_legacy_forward"]:
        assert must in names


def test_library_exports_every_declared_symbol():
    from vosdetectron_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail("libvosdet.so not built (run __graft_entry__.build())")
    L = _lib.lib()
    for name in declared():
        assert hasattr(L, name), name
        assert name in _lib.SIGNATURES, "binding missing for %s" % name
    assert L.vd_version() == 1
    assert L.vd_status_string(2) == b"unsupported shape"


def test_host_side_argument_errors_without_gpu():
    """Validation happens before any launch, so it is testable on the host."""
    from vosdetectron_amd import _lib
    L = _lib.lib()
    # rois with 4 columns -> VD_ERR_ARG (reference returns 0 and leaves zeros)
    assert L.vd_roi_align_forward(7, 7, 0.25, 2, 1, 1, 1, 1, 1, 1, 3, 4, 1, None) == _lib.VD_ERR_ARG
    assert L.vd_nms(None, 10, 5, 0.5, None, None, None, 0, None) == _lib.VD_ERR_ARG
    assert L.vd_nms_workspace_size(1000) > 1000 * 16 * 8


def test_product_path_fails_loudly_without_library(monkeypatch, tmp_path):
    from vosdetectron_amd import _lib
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "missing.so"))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _lib.lib()


def test_miopen_db_is_a_per_process_copy():
    """The tracked MIOpen Find db is a read-only seed: a
    process that imports the package points MIOPEN_USER_DB_PATH at its own
    temporary copy, outside the repository, so MIOpen's appends never touch the
    tracked files and concurrent ranks never share one file."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k != "MIOPEN_USER_DB_PATH"}
    code = ("import os, vosdetectron_amd; d = os.environ['MIOPEN_USER_DB_PATH']; "
            "print(d); print(sorted(os.listdir(d)))")
    outs = [subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                           env=env, cwd=root, timeout=120).stdout.splitlines() for _ in range(2)]
    seed = sorted(os.listdir(os.path.join(root, "vosdetectron_amd", "miopen_db")))
    for d, names in outs:
        assert not os.path.abspath(d).startswith(root), d
        assert names == repr(seed) or eval(names) == seed
        assert not os.path.exists(d)  # removed at exit
    assert outs[0][0] != outs[1][0]
    # a child started by an importing parent inherits the parent's path
    # but not its ownership -- it seeds a copy of its own
    code = ("import os, subprocess, sys, vosdetectron_amd; print(os.environ['MIOPEN_USER_DB_PATH']); "
            "sys.stdout.flush(); subprocess.run([sys.executable, '-c', 'import os, vosdetectron_amd; "
            "print(os.environ[\\'MIOPEN_USER_DB_PATH\\'])'])")
    parent, child = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                                   env=env, cwd=root, timeout=120).stdout.splitlines()
    assert parent != child and not os.path.exists(child)
    # a child that inherited the parent's copy but set its own
    # MIOPEN_USER_DB_PATH keeps that path
    code = ("import os, subprocess, sys, vosdetectron_amd; env = dict(os.environ); "
            "env['MIOPEN_USER_DB_PATH'] = '/tmp/vosdet_own_db'; "
            "subprocess.run([sys.executable, '-c', 'import os, vosdetectron_amd; "
            "print(os.environ[\\'MIOPEN_USER_DB_PATH\\'])'], env=env)")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                         env=env, cwd=root, timeout=120).stdout.splitlines()
    assert out == ["/tmp/vosdet_own_db"], out


@pytest.mark.gpu
def test_gemm_plans_are_keyed_for_this_device():
    """pinned GEMM plans apply only under a '# key' line equal to the
    running device / hipBLASLt build (vd_gemm_plans_key); the shipped file carries
    the key of the MI355X image the pins were recorded on."""
    from vosdetectron_amd import _lib
    b = ctypes.create_string_buffer(256)
    _lib.check(_lib.lib().vd_gemm_plans_key(b, 256), "vd_gemm_plans_key")
    key = b.value.decode()
    assert key.startswith("gfx950 hipblaslt-"), key
    lines = open(_lib.GEMM_PLANS).read().splitlines()
    assert "# key " + key in lines, key
