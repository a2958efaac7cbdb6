"""Entry point -- same CLI and launch model as the reference's main.py.

    python main.py [--batch_size 64] [--epochs 20] [--model res] [--save_path ./test/]
                   [--gpu 7] [--print-freq 10] [--world_size 2] [new flags ...]

Spawns ``--world_size`` rank processes with ``torch.multiprocessing.spawn``
(one per GPU; RCCL over xGMI), each running the engine in
``pytorch_multiprocessing_distributed_amd.engine.train.run_rank``.  Without a
GPU the same command runs on CPU over gloo (BASELINE config 1), e.g.:

    python main.py --world_size 2 --epochs 1 --synthetic --train_samples 512
"""
import os

from pytorch_multiprocessing_distributed_amd.config import parse_args
from pytorch_multiprocessing_distributed_amd.engine.train import run_rank
from pytorch_multiprocessing_distributed_amd.launch import run_model

args = parse_args()


def main(rank, world_size):
    run_rank(rank, world_size, args)


if __name__ == "__main__":
    os.environ["PYTHONWARNINGS"] = "ignore:semaphore_tracker:UserWarning"
    run_model(main, args.world_size, save_path=args.save_path, snapshot=__file__)
