"""bench.py's GPU-side helpers on one device: the N > 1 line's weak-scaling reference (a slab
stepped as a single domain before the communicator is attached, then re-initialised) leaves the
slab run exactly as a fresh slab would run it."""
import importlib.util
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    m._imports()
    return m


def test_single_domain_reference_then_slab_run(gpu):
    from lbm_amd import cases
    import lbm_amd
    b = _bench()
    a = cases.ldc_device(32, 32, 32, z_offset=32, nz_global=96)
    ms = b.single_domain_ms(a, 5)
    assert ms > 0.0
    a.init_ldc()  # what bench.py does before attaching
    a.attach_rccl(lbm_amd.rccl_unique_id(), 0, 1)
    fresh = cases.ldc_device(32, 32, 32, z_offset=32, nz_global=96)
    fresh.attach_rccl(lbm_amd.rccl_unique_id(), 0, 1)
    ha, hf = a.step(12), fresh.step(12)
    assert np.array_equal(ha.view(np.uint32), hf.view(np.uint32))
    for x, y in zip(a.macros(), fresh.macros()):
        assert np.array_equal(x.view(np.uint32), y.view(np.uint32))
    a.close()
    fresh.close()
