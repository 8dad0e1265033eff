"""Host side of the device window builder (lp/gpu_builder.py): the specs it ships describe the same packed layout and
objective constants as the host builder; unsupported window kinds are refused (they keep the host builder).  The
device expansion itself is compared bit for bit in tests/test_gpu_builder.py."""
import numpy as np
import pytest

from dervet_hip.lp import builder, gpu_builder, scenarios


def test_spec_layout_and_constants_match_the_host_builder():
    host, spec = scenarios.config4(range(6)), scenarios.config4(range(6), spec=True)
    pb = builder.pack_groups(host)
    desc, sz = gpu_builder.desc_of(spec)
    assert np.array_equal(desc, pb.desc)
    assert sz == dict(rows=len(pb.indptr), nnz=len(pb.indices), n=len(pb.c), m=len(pb.q))
    assert np.array_equal(np.concatenate([s.c0 for s in spec]), pb.c0)
    for s, g in zip(spec, host):
        assert (s.G, s.n, s.m) == (g.G, g.n, g.m)


def test_spec_refuses_window_kinds_the_device_builder_lacks():
    bat = scenarios.template_battery()
    with pytest.raises(NotImplementedError):
        gpu_builder.battery_group_spec(24, 1.0, np.zeros((1, 24)), bat, pv_curtail_max=np.ones((1, 24)))
    with pytest.raises(NotImplementedError):
        gpu_builder.battery_group_spec(24, 1.0, np.zeros((1, 24)), bat, grid_charge=False)
