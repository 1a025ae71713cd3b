"""Shared test setup.

Markers: ``gpu`` tests need a gfx950 device and call the product through the
C ABI (libkzgx.so); everything else runs on CPU.  The oracle (oracle/) is
imported here only as the checker."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("oracle", os.path.join("kzg-commitments_amd", "python")):
    p = os.path.join(ROOT, sub)
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and libkzgx.so")


@pytest.fixture(scope="session")
def oracle_c():
    import corc
    corc.build()
    return corc


@pytest.fixture(scope="session")
def ctx_factory():
    import kzgx
    made = {}

    def get(curve="BN254"):
        if curve not in made:
            made[curve] = kzgx.Context(curve)
            # the parity tests built on this factory target the table-less
            # Pippenger path: MSMs would otherwise take the default table
            # (tests/test_gpu_default_table.py covers that)
            made[curve].set_default_table(0)
        return made[curve]

    yield get
    for c in made.values():
        c.close()
