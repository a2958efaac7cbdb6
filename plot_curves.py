"""``plot_curves`` compatibility module: ``draw_plot(save_path)`` writes
test_accuracy.png and loss.png from train.log / test.log."""
from pytorch_multiprocessing_distributed_amd.utils.plot import draw_plot  # noqa: F401
