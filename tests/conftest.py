import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_report_header(config):
    # which library the run is testing: the build id is the hash of the sources
    try:
        from opticalflowfromdepth_amd import _native, build
        return f"libofd_fw build id {_native.build_id()} (sources {build.source_hash()})"
    except Exception as e:  # noqa: BLE001 -- a header must never fail the run
        return f"libofd_fw not loaded: {e}"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")


def load_golden(name):
    import numpy as np
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def golden_cases(npz):
    """Group 'case/field' keys of a fixture into {case: {field: array}}."""
    cases = {}
    for k in npz.files:
        if "/" in k:
            c, f = k.split("/", 1)
            cases.setdefault(c, {})[f] = npz[k]
    return cases


@pytest.fixture(scope="session")
def cuda_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")
