"""Command-line flags.

The first seven flags are the reference's, verbatim (names, defaults, help;
main.py:21-30).  The rest are new capabilities.
"""
from __future__ import annotations

import argparse


def build_parser():
    p = argparse.ArgumentParser(description="MI355X-native multiprocess data-parallel trainer")
    # ---- reference flags (main.py:22-28)
    p.add_argument("--batch_size", default=64, type=int, help="Batch size (global)")
    p.add_argument("--epochs", default=20, type=int, help="Total number of epochs to run")
    p.add_argument("--model", default="res", type=str,
                   help="Model: res (=ResNet18 [1,1,1,1] as in the reference), resnet18, "
                        "resnet18full, resnet34, resnet50, resnet101, resnet152")
    p.add_argument("--save_path", default="./test/", type=str, help="Savefiles directory")
    p.add_argument("--gpu", default="7", type=str,
                   help="kept for CLI compatibility; rank r always uses local GPU r (as in the reference)")
    p.add_argument("--print-freq", "-p", default=10, type=int, metavar="N",
                   help="print frequency (default: 10)")
    p.add_argument("--world_size", default=2, type=int, help="Gpu use number")
    # ---- new flags
    p.add_argument("--stem", "--arch", dest="stem", default="cifar", choices=["cifar", "imagenet"])
    p.add_argument("--image_size", default=None, type=int, help="input size (32 cifar / 224 imagenet)")
    p.add_argument("--num_classes", default=None, type=int, help="10 cifar / 1000 imagenet")
    p.add_argument("--dtype", default="auto", choices=["auto", "bf16", "fp32", "fp8"],
                   help="activation dtype (auto: bf16 on GPU, fp32 on CPU); fp8 = every block conv's "
                        "forward, data gradient and weight gradient on the scaled fp8 MFMA (e4m3 "
                        "weights/activations, e5m2 gradients, delayed per-tensor scaling), stem, "
                        "classifier and BatchNorm in bf16/fp32 (GPU only)")
    p.add_argument("--backend", default="auto", choices=["auto", "nccl", "rccl", "gloo"],
                   help="auto: RCCL (torch 'nccl') with GPUs, gloo on CPU")
    p.add_argument("--device", default="auto", choices=["auto", "cuda", "cpu"])
    p.add_argument("--data_root", default="./cifar10_data", type=str)
    p.add_argument("--synthetic", action="store_true", help="synthetic data of the dataset's shape")
    p.add_argument("--train_samples", default=None, type=int, help="limit dataset size")
    p.add_argument("--steps_per_epoch", default=100, type=int, help="synthetic ImageNet steps/epoch")
    p.add_argument("--max_steps", default=None, type=int, help="cap batches per epoch")
    p.add_argument("--eval_batches", default=None, type=int, help="cap eval batches")
    p.add_argument("--bucket_mb", default=25.0, type=float)
    p.add_argument("--first_bucket_mb", default=1.0, type=float)
    p.add_argument("--sync_bn", default="on", choices=["on", "off"])
    p.add_argument("--broadcast_buffers", action="store_true",
                   help="re-broadcast BN buffers from rank 0 each forward (reference DDP default)")
    p.add_argument("--lr", default=0.1, type=float)
    p.add_argument("--momentum", default=0.9, type=float)
    p.add_argument("--wd", default=1e-4, type=float)
    p.add_argument("--milestones", default="60,80", type=str)
    p.add_argument("--gamma", default=0.1, type=float)
    p.add_argument("--seed", default=None, type=int, help="seed model init on every rank")
    p.add_argument("--master_addr", default=None, type=str)
    p.add_argument("--master_port", default=None, type=int)
    p.add_argument("--resume", default="", type=str, help="resume checkpoint path")
    p.add_argument("--resume_every", default=0, type=int, help="write resume.pth every N epochs")
    p.add_argument("--compat_metrics", action="store_true",
                   help="report test accuracy like the reference (local correct / global size)")
    p.add_argument("--fixed_order", action="store_true",
                   help="never advance the sampler epoch (reference never calls set_epoch)")
    p.add_argument("--no_plot", action="store_true")
    p.add_argument("--timeout_min", default=30, type=int, help="collective timeout (minutes)")
    p.add_argument("--syncbn_comm", default="auto", choices=["auto", "xgmi", "rccl"],
                   help="SyncBN statistics transport: one-shot xGMI IPC kernel or the process "
                        "group (auto: xgmi on multi-GPU runs)")
    p.add_argument("--tune_table", default="", type=str,
                   help="per-shape kernel tuning table (JSON, ops/tuning.py) loaded before training; "
                        "default: the committed table for this device; 'online': autotune in step 0")
    p.add_argument("--save_tune_table", default="", type=str,
                   help="rank 0 writes the tuning table after the first training step")
    p.add_argument("--reducer", default="native", choices=["native", "python"],
                   help="gradient bucket reducer implementation")
    p.add_argument("--grad_compress", default="none", choices=["none", "bf16"],
                   help="wire dtype of the gradient all-reduce")
    p.add_argument("--comm", default="auto", choices=["auto", "c10d", "rccl"],
                   help="gradient-bucket transport: auto (default) = the framework's own RCCL "
                        "communicator (csrc/runtime/rccl_comm.cpp) when it can be the only in-step "
                        "communicator (SyncBN on the xGMI kernel or off) and its startup self-test "
                        "passes, else torch ProcessGroupNCCL (c10d); the choice is printed")
    p.add_argument("--step_mode", default="auto", choices=["auto", "two_stream", "one_stream", "graph"],
                   help="GPU step schedule: two_stream = weight gradients on a side HIP stream (the "
                        "device-bound large steps, e.g. ImageNet bs256); one_stream = everything on one "
                        "stream (host-bound small steps: fewer host-side forks/joins); graph = one "
                        "stream, captured once as a HIP graph and replayed (single GPU, bf16); auto: "
                        "graph for W=1 small steps, one_stream for W>1 small steps, two_stream otherwise "
                        "(small = image <= 64, e.g. the reference's CIFAR-10 ResNet18)")
    p.add_argument("--last_bucket_mb", default=2.0, type=float,
                   help="cap of the LAST gradient bucket (earliest layers: its all-reduce is "
                        "launched at the end of backward, fully exposed)")
    return p


def finalize(args):
    if args.backend == "rccl":
        args.backend = "nccl"
    if args.image_size is None:
        args.image_size = 224 if args.stem == "imagenet" else 32
    if args.num_classes is None:
        args.num_classes = 1000 if args.stem == "imagenet" else 10
    args.milestone_list = [int(m) for m in args.milestones.split(",") if m.strip()]
    return args


def parse_args(argv=None):
    return finalize(build_parser().parse_args(argv))
