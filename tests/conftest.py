import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "dect-nr-plus-sdr_amd"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libdnrp.so on the device)")
    # the C-ABI library and the oracle are built in-tree (__graft_entry__.build()); build them here
    # too when a fresh checkout runs the tests directly
    for d, so in (("dect-nr-plus-sdr_amd", "libdnrp.so"), ("oracle", "liboracle.so")):
        if not os.path.exists(os.path.join(ROOT, d, so)):
            subprocess.run(["make", "-C", os.path.join(ROOT, d), "-j8"], check=True, stdout=subprocess.DEVNULL)
