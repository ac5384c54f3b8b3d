import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run via gpurun")
    config.addinivalue_line("markers", "slow: long CPU test")


# Run order: the oracle / golden-fixture parity tests first, so that an infrastructure test (graph replay,
# RCCL-in-graph probe, CLI pipeline) failing under ``-x`` can never hide them; then the kernel-level checks;
# the whole-step graph tests last.
_ORDER = ["test_oracle_golden", "test_parity_gpu", "test_fullshape_gpu", "test_pruned_gpu", "test_wavlm_gpu",
          "test_ops_gpu", "test_stochastic_gpu", "test_gemm_gpu", "test_cli_gpu", "test_graph_gpu"]


def pytest_collection_modifyitems(session, config, items):
    def rank(item):
        stem = Path(str(item.fspath)).stem
        return _ORDER.index(stem) if stem in _ORDER else len(_ORDER) // 2
    items.sort(key=rank)      # stable: the order inside a file is kept
