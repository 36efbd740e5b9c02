import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); runs on the GPU box")
    config.addinivalue_line("markers", "slow: full-size (BASELINE) shapes")


# One summary line per BASELINE config and per hot-path parity family, so the
# tail of a run's log says which configs ran the HIP path against the oracle.
# (label, test-file stem, test-function prefixes); first match wins.
FAMILIES = [
    ("configs[0] helloworld + 2 loopback PS processes (1K x 64)", "test_libgeeps",
     ("test_reference_helloworld_runs_unchanged", "test_two_processes_loopback_bsp")),
    ("configs[1] 1M x 1024, 2 clients, full size vs oracle/torch", "test_gpu_parity",
     ("test_full_size_config1_two_clients",)),
    ("configs[2] rehearsal: libgeeps one process per GPU, cross-GPU paths forced, on one GPU",
     "test_libgeeps", ("test_one_process_per_gpu_rehearsal",)),
    ("configs[2] on real ranks: RCCL exchange + HIP sum (nccl ranks; skips below 2 GPUs)", "test_rccl",
     ("test_rccl_",)),
    ("configs[2] rehearsal, NOT RCCL: gloo exchange at 2/8 ranks around the HIP sum on one GPU "
     "(+ bench.exchange_check on the ranks; oracle-apply cases on CPU)", "test_rccl", ("test_gloo_",)),
    ("configs[2] 8 shards: RCCL-shaped exchange (gloo ranks) + one process per GPU", "",
     ("test_sharded_reduction", "test_bench_multirank_flow", "test_one_process_per_gpu",
      "test_world_one_is_local", "test_hosting_requires_divisible_clients",
      "test_rank0_runs_the_leg", "test_world_one_and_other_backends", "test_leg_")),
    ("configs[3] Inception CIFAR-10 table, 2 workers", "test_libgeeps",
     ("test_config4_inception_cifar_two_workers",)),
    ("configs[4] AlexNet table, 8 workers x 8 shards, staleness 1", "test_libgeeps",
     ("test_config5_alexnet", "test_alexnet_table_size")),
    ("north star: 8-way 1M x 1024 sum, full size vs oracle/torch", "test_gpu_parity",
     ("test_full_size_8way_bucket_sum",)),
    ("bucket sum (server apply_updates) vs oracle", "test_gpu_parity",
     ("test_bucket_sum", "test_golden_bucket", "test_gpu_add_and_zero", "test_sum_past_the_reference")),
    ("row ops, unplanned C-ABI (add_rows_from_double_index_gpu ...) vs oracle", "test_gpu_parity",
     ("test_rowop", "test_golden_rowops", "test_scatter_init", "test_segmented", "test_side_stream",
      "test_out_of_range", "test_empty_calls", "test_full_size_scatter_add", "test_unplanned",
      "test_row_ops_past_the_reference")),
    ("row / gather plans (libgeeps Update / Read) vs oracle", "test_gpu_parity",
     ("test_row_plan", "test_gather_plan")),
    ("C-ABI from C99 vs oracle", "test_gpu_parity", ("test_c_abi_consumer",)),
    ("IPC buffers between processes through the C-ABI (tagged mappings)", "test_ipc", ("test_",)),
    ("IPC audit: the runtime's mis-mappings re-derived from the committed round-6 logs (CPU)", "test_ipc_audit",
     ("test_",)),
    ("libgeeps end to end (other process / consistency cases)", "test_libgeeps", ("test_",)),
    ("wire path: libgeeps ZMTP/3.0 ROUTER vs a stock libzmq ROUTER (CPU)", "test_zmtp", ("test_",)),
    ("host-tier row ops (a4: add_rows_from_double_index_cpu ...) vs oracle (CPU)", "test_host_rows", ("test_",)),
    ("host tier's shared oplogs: a peer process maps and checks them", "test_hostshare", ("test_",)),
    ("oracle vs golden vectors + layout vs reference headers (CPU)", "", ("test_",)),
]
_family_counts = {}


def _family(nodeid: str) -> str:
    path, _, name = nodeid.partition("::")
    stem = os.path.splitext(os.path.basename(path))[0]
    for label, file_stem, prefixes in FAMILIES:
        if file_stem and file_stem != stem:
            continue
        if not file_stem and label.startswith("oracle") and stem not in ("test_oracle", "test_layout"):
            continue
        if any(name.startswith(p) for p in prefixes):
            return label
    return "other (ABI, schedule, host logic)"


def pytest_runtest_logreport(report):
    if report.when == "call" or (report.when == "setup" and report.outcome != "passed"):
        c = _family_counts.setdefault(_family(report.nodeid), {"passed": 0, "failed": 0, "skipped": 0})
        c[report.outcome] = c.get(report.outcome, 0) + 1


def pytest_terminal_summary(terminalreporter):
    if not _family_counts:
        return
    tr = terminalreporter
    tr.section("geeps parity summary (per BASELINE config / hot-path family)")
    order = [f[0] for f in FAMILIES] + ["other (ABI, schedule, host logic)"]
    for label in order:
        c = _family_counts.get(label)
        if c:
            tr.write_line(f"{label}: {c['passed']} passed, {c['failed']} failed, {c['skipped']} skipped")


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import geeps_amd
    geeps_amd.lib()  # the HIP library must load: no fallback
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def golden_rowops():
    import numpy as np
    return np.load(os.path.join(GOLDEN, "rowops.npz"))


@pytest.fixture(scope="session")
def golden_bucket():
    import numpy as np
    return np.load(os.path.join(GOLDEN, "bucket.npz"))


@pytest.fixture(scope="session")
def manifest():
    import json
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)
