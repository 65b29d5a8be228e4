"""Epoch-loss history — drop-in for the reference utils/callbacks.py:7-49
(host bookkeeping: a text log plus a loss curve png; matplotlib and scipy are
optional here and the png is skipped without them)."""
import datetime
import os


class LossHistory:
    def __init__(self, log_dir):
        self.log_dir = log_dir
        self.time_str = datetime.datetime.strftime(datetime.datetime.now(), "%Y_%m_%d_%H_%M_%S")
        self.save_path = os.path.join(self.log_dir, "loss_" + str(self.time_str))
        self.losses = []
        os.makedirs(self.save_path)

    def append_loss(self, loss):
        self.losses.append(loss)
        with open(os.path.join(self.save_path, "epoch_loss_" + str(self.time_str) + ".txt"),
                  "a") as f:
            f.write(str(loss))
            f.write("\n")
        self.loss_plot()

    def loss_plot(self):
        try:
            import matplotlib
            matplotlib.use("Agg")
            from matplotlib import pyplot as plt
        except ImportError:
            return
        iters = range(len(self.losses))
        plt.figure()
        plt.plot(iters, self.losses, "red", linewidth=2, label="train loss")
        try:
            import scipy.signal
            num = 5 if len(self.losses) < 25 else 15
            plt.plot(iters, scipy.signal.savgol_filter(self.losses, num, 3), "green",
                     linestyle="--", linewidth=2, label="smooth train loss")
        except Exception:  # too few points for the filter, as the reference tolerates
            pass
        plt.grid(True)
        plt.xlabel("Epoch")
        plt.ylabel("Loss")
        plt.legend(loc="upper right")
        plt.savefig(os.path.join(self.save_path, "epoch_loss_" + str(self.time_str) + ".png"))
        plt.cla()
        plt.close("all")
