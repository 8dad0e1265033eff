"""The result all-gather inside the library: dvh_comm_init +
dvh_gather_results over the library's own RCCL communicator.  One GPU on the test box, so world size 1: the gathered
rows must equal parallel.result_rows bit for bit, in a process where PyTorch's own RCCL is loaded and initialised as
well (the two copies must not interfere), and the torch.distributed gather of the same rows must agree.  The N > 1
logic (tags, shards, overlap) is covered by the gloo tests in tests/test_distributed.py."""
import socket

import numpy as np
import pytest
import torch

from dervet_hip import BatchSolver, parallel
from dervet_hip.lp import builder, scenarios

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_library_gather_world_one_returns_the_result_rows():
    import torch.distributed as dist
    groups = scenarios.config4(range(8))
    pb = builder.pack_groups(groups)
    dev = pb.to_torch("cuda:0").alloc_outputs()
    tags = parallel.tag_array([t for g in groups for t in g.tags])
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        with BatchSolver(0) as s:
            s.solve_packed(dev)
            desc = np.asarray(pb.desc)
            runs = parallel.dispatch_runs(desc)
            tmax = max(r[4] for r in runs)
            rows = parallel.result_rows(dev.stats, dev.istats, dev.x, desc, tmax, runs,
                                        tags=torch.as_tensor(tags, device="cuda:0"))
            g = parallel.LibraryGather.from_torch(s)
            assert s.comm_info() == (0, 1)
            out = g.gather(rows)
            torch.cuda.synchronize()
            assert out.shape == rows.shape and torch.equal(out, rows)
            # asynchronous form, then the torch.distributed gather of the same rows
            pend = g.gather(rows, async_op=True)
            out2 = pend.wait()
            assert torch.equal(out2, rows)
            ref = parallel.gather_rows(rows, counts=[rows.shape[0]])
            assert torch.equal(ref, out)
            r = parallel.by_tag(parallel.rows_to_numpy(out))
            assert (r["status"] == 0).all() and len(r["obj"]) == 96
    finally:
        dist.destroy_process_group()


def test_comm_errors_are_codes():
    with BatchSolver(0) as s:
        with pytest.raises(Exception, match="no communicator"):
            s.gather_results(torch.zeros(4, device="cuda:0"), torch.zeros(4, device="cuda:0"))
        with pytest.raises(ValueError):
            s.comm_init(0, 1, b"short")
