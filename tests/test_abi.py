"""CPU checks of the C-ABI library: it loads and exports every symbol include/ngp_hip.h declares."""
import os
import re

import ngp_abi as A

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "ngp_hip.h")).read()
    return sorted(set(re.findall(r"^(?:ngp_status|const char\*)\s+(ngp_\w+)\(", src, re.M)))


def test_header_declares_expected_entry_points():
    syms = declared_symbols()
    for s in ("ngp_model_create", "ngp_model_infer", "ngp_train_step", "ngp_density_grid_update", "ngp_render"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    lib = A.load()
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    assert set(declared_symbols()) <= set(A.EXPORTS)
    assert lib.ngp_version().decode().startswith("ngp_hip")


def test_invalid_config_reports_error_without_gpu_work():
    import ctypes as C
    lib = A.load()
    cfg = A.default_config(F=3)
    h = C.c_void_p()
    st = lib.ngp_model_create(0, C.byref(cfg), 1337, C.byref(h))
    assert st != 0
    assert "n_features_per_level" in lib.ngp_last_error().decode()
