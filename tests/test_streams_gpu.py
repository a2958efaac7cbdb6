"""Step streams (ops/functional.py::init_step_streams): three distinct new HIP streams at the
step priority, the main one made current, the weight-gradient side stream and the gradient-
collective stream registered for their users, idempotent per device; RcclComm runs on the
pre-created collective stream when given its handle (profiles/queues_r04.txt)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_init_step_streams_distinct_and_idempotent():
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    dev = torch.device("cuda", 0)
    before = torch.cuda.current_stream(dev)
    try:
        main = OF.init_step_streams(dev)
        assert torch.cuda.current_stream(dev).cuda_stream == main.cuda_stream
        e = OF._STEP_STREAMS[dev]
        handles = {e["main"].cuda_stream, e["wgrad"].cuda_stream, e["comm"].cuda_stream}
        assert len(handles) == 3 and 0 not in handles
        assert OF._wgrad_stream(dev).cuda_stream == e["wgrad"].cuda_stream
        assert OF.comm_stream_handle(dev) == e["comm"].cuda_stream
        # idempotent: same streams, main made current again
        torch.cuda.set_stream(before)
        assert OF.init_step_streams(dev).cuda_stream == main.cuda_stream
        assert torch.cuda.current_stream(dev).cuda_stream == main.cuda_stream
        # work on the step streams runs and orders like on any stream
        x = torch.arange(1 << 16, device=dev, dtype=torch.float32)
        with torch.cuda.stream(e["wgrad"]):
            e["wgrad"].wait_stream(main)
            y = x * 2
        main.wait_stream(e["wgrad"])
        assert torch.equal(y, x * 2)
    finally:
        torch.cuda.set_stream(before)


def test_rccl_comm_on_precreated_stream():
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    from pytorch_multiprocessing_distributed_amd.parallel import rccl
    dev = torch.device("cuda", 0)
    before = torch.cuda.current_stream(dev)
    try:
        OF.init_step_streams(dev)
        h = OF.comm_stream_handle(dev)
        c = rccl.register(C.RcclComm(bytes(C.RcclComm.unique_id()), 0, 1, 0, OF.STREAM_PRIO, h))
        assert c.stream_handle == h
        t = torch.arange(4097, device=dev, dtype=torch.float32)
        ref = t.clone()
        c.all_reduce_(t, 0)
        torch.cuda.synchronize()
        assert torch.equal(t, ref) and c.check()
        del c                      # does not destroy the borrowed stream
        z = torch.ones(8, device=dev)
        with torch.cuda.stream(OF._STEP_STREAMS[dev]["comm"]):
            z.mul_(3)
        torch.cuda.synchronize()
        assert torch.equal(z, torch.full((8,), 3.0, device=dev))
    finally:
        torch.cuda.set_stream(before)
