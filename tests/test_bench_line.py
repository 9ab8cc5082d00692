"""bench.py's printed line (CPU only): the driver keeps only the tail of
stdout, so the JSON line must stay short enough to survive whole while
carrying every BASELINE config (C1500, C64, CMIX with M6 beside it, IMIX,
JMIX), the end-to-end rates and, with N > 1, the checked all-gather.  The
full result is built from the round-4 closing tree's committed line
(profiles/r04/final_v25/bench_final.json) plus worst-case additions (8
ranks, an all-gather report, the e2e key)."""
import copy
import json
import os

from conftest import ROOT

import bench


def _full(n_gpus=1):
    with open(os.path.join(ROOT, "profiles", "r04", "final_v25", "bench_final.json")) as f:
        full = json.loads([x for x in f if x.startswith("{")][-1])
    full = copy.deepcopy(full)
    full["secondary"]["cmix"]["m6"] = {"kernel_ms": 2.5123, "same_records": True, "frac": 0.6543}
    full["e2e"] = {"pcie_h2d_gbs": 56.71, "gather_threads": 8,
                   "c1500": {"mpkts": 36.12, "path": "staged", "frame_gbs": 54.18, "of_pcie": 0.955,
                             "frames": 1048576, "records": "copied", "staged_mpkts": 36.12,
                             "ring_mpkts": 31.9},
                   "c64": {"mpkts": 448.12, "path": "ring", "frame_gbs": 28.68, "of_pcie": 0.506,
                           "frames": 4194304, "records": "registered", "staged_mpkts": 121.5,
                           "ring_mpkts": 448.12},
                   "c64_rec32": {"mpkts": 776.2, "path": "ring", "frame_gbs": 49.68,
                                 "of_pcie": 0.878, "frames": 4194304,
                                 "records": "registered 32 B", "staged_mpkts": 589.16,
                                 "ring_mpkts": 776.2},
                   "scrub_wait_s": 0.07, "numa": {"node": 0, "cpus": 128}}
    if n_gpus > 1:
        full["n_gpus"] = n_gpus
        full["config"]["rccl_ranks"] = n_gpus
        full["per_rank_kernel_ms"] = [4.1234] * n_gpus
        full["value_no_gather"] = 33333.3
        full["allgather"] = {
            "bytes_per_rank": 134217728, "ms": 1.2345, "algbw_gbs": 869.6, "busbw_gbs": 760.9,
            "rccl_ranks": n_gpus, "overlap_loss": 0.0712,
            "buffer_placement": {"alloc": "pptk_rx_gather_alloc", "candidates": 8, "chosen": 3,
                                 "chosen_ms": 4.6123, "first_ms": 5.1234,
                                 "freed_bytes": 123456789012, "settle_ms": 0},
            "gathered_check": {"own_slice_equals_records": True, "sampled_frames": 32768,
                               "sampled_frames_per_rank": 4096, "sampled_mismatches": 0}}
    return full


def test_line_fits_the_stored_tail_and_carries_every_config():
    for n in (1, 8):
        line = bench.compact_line(_full(n), detail_path="gpurun_out/bench_detail.json")
        text = json.dumps(line)
        assert len(text) < bench.LINE_MAX_CHARS, (n, len(text))
        # what the driver's tail must show: C64's and CMIX's value, kernel
        # time and read-roofline fraction, beside the primary's
        tail = text[-bench.LINE_MAX_CHARS:]
        back = json.loads(tail)
        for cfg in ("c1500", "c64", "cmix", "imix", "jmix", "c1500_rec32", "c64_rec32"):
            e = back["configs"][cfg]
            assert all(isinstance(e[k], (int, float)) for k in ("mpkts", "kernel_ms", "frac")), cfg
        assert back["configs"]["cmix"]["m6_ms"] == 2.5123
        assert back["e2e"]["c1500"]["mpkts"] == 36.12
        assert back["e2e"]["c64_rec32"]["of_pcie"] == 0.878   # the compact host path
        assert "numa" not in back["e2e"] and "scrub_wait_s" not in back["e2e"]
        for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                  "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
                  "roofline", "cpu_baseline"):
            assert k in back, k
        assert back["roofline"]["frac"] == _full()["roofline"]["frac"]
        assert back["cpu_baseline"]["cores"] == _full()["cpu_baseline"]["cores"]


def test_compact_multigpu_line_passes_validation():
    line = bench.compact_line(_full(8))
    assert bench.validate_line(line) == []
    bad = copy.deepcopy(line)
    bad["allgather"]["gathered_check"]["sampled_mismatches"] = 3
    assert bench.validate_line(bad)
