"""--step_mode resolution (engine/train.py resolve_step_mode): the device-bound ImageNet step keeps
the two-stream schedule, the host-bound CIFAR-size step runs on one stream, captured as a HIP graph
when there is one process."""
from pytorch_multiprocessing_distributed_amd.engine.train import resolve_step_mode


def test_auto_modes():
    assert resolve_step_mode("auto", 1, True, 224, "bf16") == "two_stream"
    assert resolve_step_mode("auto", 8, True, 224, "bf16") == "two_stream"
    assert resolve_step_mode("auto", 1, True, 32, "bf16") == "graph"
    assert resolve_step_mode("auto", 2, True, 32, "bf16") == "one_stream"
    assert resolve_step_mode("auto", 1, False, 32, "fp32") == "two_stream"      # CPU: no streams


def test_graph_needs_one_process_and_bf16():
    assert resolve_step_mode("graph", 2, True, 32, "bf16") == "one_stream"
    assert resolve_step_mode("graph", 1, True, 32, "fp8") == "one_stream"
    assert resolve_step_mode("graph", 1, True, 224, "bf16") == "graph"        # explicit request
    assert resolve_step_mode("one_stream", 1, True, 224, "bf16") == "one_stream"
