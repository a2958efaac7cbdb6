"""Training curves from the text logs (reference plot_curves.py:7-37):
``test_accuracy.png`` (train vs test accuracy) and ``loss.png``."""
from __future__ import annotations

import os

from .logger import Logger


def draw_plot(save_path):
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    train_log = Logger(os.path.join(save_path, "train.log")).read()
    test_log = Logger(os.path.join(save_path, "test.log")).read()
    epoch, train_loss, train_acc = zip(*[row[:3] for row in train_log])
    epoch_t, test_loss, test_acc = zip(*[row[:3] for row in test_log])

    plt.plot(epoch, train_acc, "-b", label="train")
    plt.plot(epoch_t, test_acc, "-r", label="test")
    plt.xlabel("Epoch")
    plt.ylabel("accuracy")
    plt.legend(loc="lower right")
    plt.title("TEST accuracy ")
    plt.savefig(os.path.join(save_path, "test_accuracy.png"))
    plt.close()

    plt.plot(epoch, train_loss, "-b", label="train")
    plt.plot(epoch_t, test_loss, "-r", label="test")
    plt.xlabel("Epoch")
    plt.ylabel("loss")
    plt.legend(loc="upper right")
    plt.title("loss")
    plt.savefig(os.path.join(save_path, "loss.png"))
    plt.close()
