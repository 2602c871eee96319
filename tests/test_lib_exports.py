"""The C-ABI library loads on the CPU host and exports every entry point include/otslam.h declares, and the
ctypes table binds exactly that set (no compute call — no GPU here)."""
import ctypes as C
import os
import re

from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "otslam.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ot_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_core_entry_points():
    names = _declared()
    for n in ("ot_tsdf_create", "ot_tsdf_integrate", "ot_unproject", "ot_voxel_down_sample",
              "ot_remove_statistical_outlier", "ot_remove_radius_outlier", "ot_tsdf_extract_triangle_mesh"):
        assert n in names


def test_library_exports_every_declared_symbol(pkg):
    lib = C.CDLL(pkg._lib.LIB_PATH)
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, f"libotslam_hip.so lacks {missing}"


def test_ctypes_table_matches_header(pkg):
    assert sorted(pkg._lib.SIGNATURES) == _declared()
    lib = pkg.native_library()
    assert not lib._ot_missing
    assert lib.ot_abi_version() == 1
    assert b"gfx950" in lib.ot_version()


def test_library_is_the_build_of_these_sources(pkg):
    """VERDICT r3 'next' 1: the source hash is compiled into the library (ot_version) and equals the hash of the
    sources beside it; a library built from other sources is refused at load."""
    L = pkg._lib
    lib = pkg.native_library()
    assert L.library_source_hash(lib) == L.source_hash()
    import importlib

    sh = importlib.import_module(pkg.__name__ + "._srchash")
    saved_lib, saved_compute = L._lib, sh.compute
    try:
        L._lib = None
        sh.compute = lambda *a: "0123456789abcdef"  # as if a source changed after the build
        import pytest

        with pytest.raises(RuntimeError, match="stale HIP library"):
            L.load()
    finally:
        sh.compute = saved_compute
        L._lib = saved_lib


def test_makefile_hash_matches_package_hash(pkg):
    """The Makefile's hash (python3 _srchash.py) is the package's source_hash()."""
    import subprocess
    import sys

    out = subprocess.run([sys.executable, os.path.join(os.path.dirname(pkg._lib.LIB_PATH), "_srchash.py")],
                         capture_output=True, text=True, check=True).stdout.strip()
    assert out == pkg._lib.source_hash()


def test_error_path_without_device(pkg):
    """Argument validation happens before any device work: a NULL handle is rejected with a message."""
    lib = pkg.native_library()
    st = lib.ot_tsdf_reset(None)
    assert st == pkg._lib.OT_ERR_INVALID_ARGUMENT
    assert b"ScalableTSDFVolume" in lib.ot_last_error()
