import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")

# Collection order of the modules: the oracle-parity modules run first, the CLI / multi-process
# plumbing last, so that under `pytest -x` a plumbing failure can never hide the parity evidence.  Modules not
# named keep their place between the two groups.
_FIRST = ["test_oracle_golden.py", "test_native_abi.py", "test_gpu_parity.py", "test_gpu_dnn_configs.py",
          "test_gpu_dnn.py"]
_LAST = ["test_sharding_gloo.py", "test_gpu_cli.py"]


def _module_rank(item) -> int:
    name = os.path.basename(str(item.fspath))
    if name in _FIRST:
        return _FIRST.index(name)
    if name in _LAST:
        return 100 + _LAST.index(name)
    return 50


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def pytest_collection_modifyitems(session, config, items):
    # stable sort: the order of the tests inside a module is unchanged
    items.sort(key=_module_rank)


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
