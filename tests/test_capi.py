"""The C-ABI library loads and exports every symbol include/yacht_hip.h declares (no GPU)."""
import ctypes
import os
import re

import yacht_amd
from conftest import REPO


def declared_functions():
    src = open(os.path.join(REPO, "include", "yacht_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(yk_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for required in ("yk_step", "yk_valid_mask", "yk_ended", "yk_canonical", "yk_score_table", "yk_featurize",
                     "yk_net_predict", "yk_net_leaf_prior", "yk_selfplay", "yk_mcts_search", "yk_engine_pack_records", "yk_arena", "yk_greedy_action",
                     "yk_arena_results"):
        assert required in names


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(yacht_amd.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_covers_the_header():
    from yacht_amd._lib import SIGNATURES
    assert set(declared_functions()) <= set(SIGNATURES)


def test_version_and_error_entry_points():
    lib = yacht_amd.lib()
    assert lib.yk_version().startswith(b"yacht_hip")
    assert lib.yk_last_hip_error() == 0


def test_null_arguments_are_rejected_without_a_gpu():
    lib = yacht_amd.lib()
    assert lib.yk_step(None, None, None, 0, None, None, None, None, None, 4, None) == -1
    assert lib.yk_valid_mask(None, None, None, None, 1, None) == -1
    assert lib.yk_engine_create(None, None, None) == -1
    assert lib.yk_arena(None, 0, 0, None, 0, 1, None) == -1
    assert lib.yk_greedy_action(None, None, 1, None) == -1
    assert lib.yk_arena_results(None, None, None, None, None, None, None) == -1
    for f in ("yk_net_predict", "yk_net_predict_features", "yk_net_leaf_prior"):
        assert getattr(lib, f)(None, None, None, None, 1, None) == -1
    assert lib.yk_step(None, None, None, 0, None, None, None, None, None, 0, None) == 0  # empty batch
