"""fp8 conv-selection policy (ops/functional.py::fp8_eligible): which ResNet-50 block
convs run their forward in fp8 under each PMD_FP8_CONVS policy (host logic only)."""
import pytest

from pytorch_multiprocessing_distributed_amd.models import ResNet50
from pytorch_multiprocessing_distributed_amd.ops import functional as OF


def _block_convs(m):
    return [mod for mod in m.modules() if getattr(mod, "weight", None) is not None
            and mod.weight.dim() == 4 and mod is not m.conv1]


@pytest.fixture
def policy():
    saved = (OF.FP8_CONVS, OF.FP8_MIN_KG)
    yield
    OF.FP8_CONVS, OF.FP8_MIN_KG = saved


def test_spatial_policy_selects_the_3x3_convs(policy):
    OF.FP8_CONVS, OF.FP8_MIN_KG = "spatial", 128
    convs = _block_convs(ResNet50(num_classes=10, stem="imagenet"))
    assert len(convs) == 52
    sel = [c for c in convs if OF.fp8_eligible(c, c.weight.shape[1])]
    assert len(sel) == 16 and all(tuple(c.weight.shape[2:]) == (3, 3) for c in sel)


def test_all_policy_skips_half_empty_k_tiles(policy):
    OF.FP8_CONVS, OF.FP8_MIN_KG = "all", 128
    convs = _block_convs(ResNet50(num_classes=10, stem="imagenet"))
    sel = [c for c in convs if OF.fp8_eligible(c, c.weight.shape[1])]
    # the five layer-1 1x1 convs over 64 input channels (Kg = 64) stay bf16
    assert len(sel) == 47
    assert all(c.weight.shape[1] * c.weight.shape[2] * c.weight.shape[3] >= 128 for c in sel)
    OF.FP8_MIN_KG = 0
    assert all(OF.fp8_eligible(c, c.weight.shape[1]) for c in convs)
