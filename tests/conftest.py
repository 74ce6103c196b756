import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: longer CPU cases")


@pytest.fixture(scope="session")
def oracle_bin():
    """The clean-room CPU restatement (test infrastructure only)."""
    path = os.path.join(ROOT, "oracle", "_build", "dd_oracle")
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), os.path.join(ROOT, "oracle", "_build", "dd_oracle")],
                       capture_output=True, text=True)
    if not os.path.exists(path):
        pytest.fail("cannot build oracle/_build/dd_oracle: " + r.stderr)
    return path


@pytest.fixture(scope="session")
def native_lib():
    # build only when the library is missing: __graft_entry__.build() is the build step, and on a
    # GPU box the snapshot's file times can make every object look stale (a minute of hipcc)
    from sgufp_solver_amd import engine
    if not os.path.exists(engine.LIB_PATH):
        from sgufp_solver_amd import build
        build.build_native()
    return engine.load_library()
