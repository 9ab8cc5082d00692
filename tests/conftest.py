import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")
GOLDEN_SETS = ("edge", "fuzz", "c64", "c1500", "cmix", "icmp", "frag")
# the product library built with -DPPTK_RX_TEST_HOOKS (Makefile "hooks"):
# the fault-injection knobs of the failure-path tests exist only there
HOOKS_LIB = os.path.join(ROOT, "tests", "hooks", "libpptkrx_hooks.so")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


def load_golden(name):
    import numpy as np
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle.oracle import Oracle, build
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        build()
    return Oracle()


@pytest.fixture(scope="session")
def reference_lib():
    from oracle.oracle import REF_SO, Reference
    if not os.path.exists(REF_SO):
        pytest.skip("oracle/_ref not built (reference tree absent)")
    return Reference()
