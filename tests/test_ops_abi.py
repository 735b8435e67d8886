"""The ctypes argument structs must match the C structs in csrc/args.h
(runs on CPU: loading the library does not need a device)."""

import ctypes as C

import pytest

from foremast_amd.ops import _native as nat
from foremast_amd.ops import build


@pytest.fixture(scope="module")
def lib():
    try:
        build.build()
    except RuntimeError as e:  # pragma: no cover
        pytest.skip(f"no HIP toolchain: {e}")
    lib = nat.load()
    if lib is None:
        pytest.skip("library failed to load")
    lib.fm_abi_sizeof.restype = C.c_longlong
    lib.fm_abi_offsetof.restype = C.c_longlong
    return lib


@pytest.mark.parametrize("name", ["DetectArgs", "SmoothArgs", "RankArgs", "WindowArgs", "BivArgs"])
def test_struct_sizes(lib, name):
    assert lib.fm_abi_sizeof(name.encode()) == C.sizeof(getattr(nat, name))


@pytest.mark.parametrize("name,field", [
    ("SmoothArgs", "det"), ("SmoothArgs", "season_out"), ("SmoothArgs", "grid"), ("SmoothArgs", "head_dev"), ("SmoothArgs", "season_hb"), ("SmoothArgs", "nvalid_out"),
    ("DetectArgs", "pw_scale"), ("DetectArgs", "app_stats"), ("DetectArgs", "ld_cur"),
    ("DetectArgs", "anom_count"), ("DetectArgs", "anom_cap"), ("DetectArgs", "thr_lut"), ("DetectArgs", "lut_n"),
    ("DetectArgs", "row_out"), ("DetectArgs", "tick_min"), ("DetectArgs", "shift_one_step"),
    ("RankArgs", "pvals"), ("RankArgs", "alpha"), ("RankArgs", "p_friedman"), ("RankArgs", "pods_b"), ("RankArgs", "z_crit"), ("WindowArgs", "det"),
    ("BivArgs", "eps"), ("BivArgs", "app_stats"),
])
def test_struct_offsets(lib, name, field):
    cls = getattr(nat, name)
    assert lib.fm_abi_offsetof(name.encode(), field.encode()) == getattr(cls, field).offset


def test_module_local_struct_sizes(lib):
    """Structs declared next to their kernels (lstm / lstm_train / decompose)."""
    from foremast_amd.ops import kernels, lstm, lstm_train, pack
    for sym, cls in (("fm_lstm_args_size", lstm.LstmArgs), ("fm_lstm_train_args_size", lstm_train.LstmTrainArgs),
                     ("fm_decompose_args_size", kernels.DecompArgs), ("fm_lstm_level_args_size", lstm.LevelArgs),
                     ("fm_hw_state_args_size", kernels.HwStateArgs),
                     ("fm_hw_update_args_size", kernels.HwUpdateArgs), ("fm_pack_args_size", pack.PackArgs)):
        f = getattr(lib, sym)
        f.restype = C.c_longlong
        assert f() == C.sizeof(cls), sym


def test_hw_seq_geometry(lib):
    """Variant 6 (hw_seq.hip) host helpers: threads per series (two grid points per thread up
    to m = 96, one at m = 144; 16..64 threads), the LDS of one workgroup (two fp32 images of
    the padded week plus a count per series) and the seasons it is instantiated for."""
    nat.load()  # argtypes / restype
    assert lib.fm_hw_seq_tpc(72, 64) == 32 and lib.fm_hw_seq_tpc(72, 16) == 16 and lib.fm_hw_seq_tpc(72, 33) == 32
    assert lib.fm_hw_seq_tpc(144, 64) == 64 and lib.fm_hw_seq_tpc(144, 5) == 32
    assert lib.fm_hw_seq_tpc(72, 65) == 0 and lib.fm_hw_seq_tpc(1440, 64) == 0 and lib.fm_hw_seq_tpc(70, 8) == 0
    assert lib.fm_hw_seq_lds_bytes(504, 72, 64) == (2 * 8 * (504 + 4) + 8) * 4
    assert lib.fm_hw_seq_lds_bytes(504, 72, 16) == (2 * 16 * (504 + 4) + 16) * 4
    none = C.c_size_t(-1).value
    assert lib.fm_hw_seq_lds_bytes(500, 72, 64) == none       # not a whole number of seasons
    assert lib.fm_hw_seq_lds_bytes(72, 72, 64) == none        # one season: nothing to fit
    assert lib.fm_hw_seq_lds_bytes(2016, 288, 64) == (2 * 4 * (2016 + 4) + 4) * 4  # one grid point per thread
