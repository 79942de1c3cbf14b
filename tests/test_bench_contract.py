"""bench.py's roofline bookkeeping on the host (no GPU): the dominant op is priced against
the ceiling its algorithmic intensity falls under, and PMC traffic per launch is attributed
from a committed per-kernel profile."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _summary(name, flops, nbytes, mean_ms=0.05, launches=10):
    return {name: dict(total_ms=mean_ms * launches, mean_ms=mean_ms, flops=flops, bytes=nbytes, launches=launches),
            "other": dict(total_ms=0.01, mean_ms=0.001, flops=0, bytes=1, launches=10)}


def test_below_ridge_is_priced_against_hbm(tmp_path):
    # 2 T N K over T (N + K) bf16 operands at T = 262144, N = 288, K = 96: ~72 FLOP/B
    T, N, K = 262144, 288, 96
    roof, table = bench.kernel_roofline(_summary("token_wgrad", 2.0 * T * N * K, T * (N + K) * 2),
                                        str(tmp_path / "none.json"))
    assert roof["bound"] == "hbm" and roof["unit"] == "GB/s" and roof["kernel"] == "token_wgrad"
    assert abs(roof["achieved"] - T * (N + K) * 2 / 0.05e-3 / 1e9) < 0.1
    assert abs(roof["frac"] - roof["achieved"] / bench.HBM_PEAK_GBS) < 1e-4
    assert roof["intensity_flop_per_byte"] < roof["ridge"] == 312.5
    assert roof["frac_other"]["bound"] == "mfma" and roof["traffic"] is None
    assert set(table) == {"token_wgrad", "other"}


def test_above_ridge_is_priced_against_mfma(tmp_path):
    T, N, K = 16384, 3072, 3072           # ~1200 FLOP/B
    roof, _ = bench.kernel_roofline(_summary("token_gemm", 2.0 * T * N * K, (T * K + T * N + N * K) * 2),
                                    str(tmp_path / "none.json"))
    assert roof["bound"] == "mfma" and roof["unit"] == "TFLOP/s"
    assert roof["intensity_flop_per_byte"] > roof["ridge"]
    assert abs(roof["frac"] - roof["achieved"] / bench.MFMA_BF16_PEAK_TFS) < 1e-5


def test_gather_kernels_stay_hbm(tmp_path):
    roof, _ = bench.kernel_roofline(_summary("msda_bwd", 1e12, 1e8), str(tmp_path / "none.json"))
    assert roof["bound"] == "hbm"


def test_pmc_traffic_sums_kernel_and_reduction_per_launch(tmp_path):
    prof = {
        "void vs::token_wgrad_kernel<256, 128, 4, 2, 3, 0>(...)": dict(dispatches=4, fetch_bytes=100.0, write_bytes=20.0),
        "void vs::token_wgrad_reduce_kernel<256, 128, 4, 2, 16>(...)": dict(dispatches=2, fetch_bytes=30.0,
                                                                             write_bytes=2.0),
        "void vs::unrelated_kernel(...)": dict(dispatches=9, fetch_bytes=1e9, write_bytes=1e9),
    }
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps(prof))
    traffic, kernels = bench.pmc_traffic("token_wgrad", str(p))
    # (4 x 120 + 2 x 32) bytes over the 4 dispatches of the first pattern
    assert traffic == int((4 * 120 + 2 * 32) / 4)
    assert kernels == ["token_wgrad_kernel<", "token_wgrad_reduce_kernel<"]
    assert bench.pmc_traffic("token_wgrad", str(tmp_path / "missing.json")) == (None, None)
