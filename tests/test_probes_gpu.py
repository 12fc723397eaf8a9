"""HIP bandwidth probes on a real MI355X."""
import pytest

pytestmark = pytest.mark.gpu


def test_hbm_probe_reasonable():
    from kgwe.agent import probes

    r = probes.probe_hbm(0, 1 << 30, 5)
    # MI355X: 8 TB/s spec, ~6.3 TB/s achievable copy (MI355X_MICROARCH.md)
    assert 2000 < r.copy_gbps < 8500, r
    assert 2000 < r.read_gbps < 8500, r
    assert 1000 < r.lds_copy_gbps < 8500, r


@pytest.mark.multigpu
def test_p2p_probe_pair():
    from kgwe.agent import probes

    bw = probes.probe_p2p(1, 0, 256 << 20, 5)
    assert bw is not None and bw > 10.0
