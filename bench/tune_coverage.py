"""Which shapes of a model does the committed tuning table NOT cover?  Loads the default
tables (ops/tables/), runs two training steps of each model at 224x224 / per-GPU batch
256, and reports how many conv / wgrad shapes were autotuned online (uncovered shapes get a
run-dependent kernel choice -- the thing the tables exist to prevent).

    python bench/tune_coverage.py resnet34 resnet18full resnet101 ...
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from pytorch_multiprocessing_distributed_amd.data.loader import SyntheticImageNet
    from pytorch_multiprocessing_distributed_amd.engine.optim import FusedSGD
    from pytorch_multiprocessing_distributed_amd.models import build_model
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.ops import tuning
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    from pytorch_multiprocessing_distributed_amd.parallel.dp import DataParallel
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    OF.init_step_streams(dev)
    for name in sys.argv[1:]:
        C.conv_autotune_clear()
        C.wgrad_autotune_clear()
        src, n0 = tuning.load_default()
        c0, w0 = len(C.conv_autotune_export()), len(C.wgrad_autotune_export())
        torch.manual_seed(0)
        model = DataParallel(build_model(name, num_classes=1000, stem="imagenet").to(dev), None)
        opt = FusedSGD(model, lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=True)
        data = SyntheticImageNet(256, 224, 1000, steps=2, device=dev, dtype=torch.bfloat16, cpad=8)
        model.train()
        for i in range(2):
            x, y = data.batch_at(i)
            loss = OF.cross_entropy(model(x), y)
            opt.zero_grad()
            loss.backward(OF.loss_seed(loss))
            opt.step()
        torch.cuda.synchronize()
        c1, w1 = len(C.conv_autotune_export()), len(C.wgrad_autotune_export())
        print(f"{name}: table {src} ({n0} entries); online-tuned conv shapes {(c1 - c0) // 14}, "
              f"wgrad shapes {(w1 - w0) // 12}", flush=True)
        del model, opt, data
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
