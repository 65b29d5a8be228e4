"""Per-epoch loss log for the training scripts' `LossHistory(log_dir)` /
`.append_loss(value)` calls (reference interface: utils/callbacks.py:7-49,
called at e.g. train_50_3_r.py:276,350).

Host bookkeeping only, out of the hot path.  Each run
gets its own directory under `log_dir`; every appended value goes to a text
file (one value per line) as soon as it arrives, and a small dependency-free
SVG chart of the curve and its running mean is rewritten beside it.
"""
import os
import time


class LossHistory:
    def __init__(self, log_dir):
        self.log_dir = log_dir
        stamp = time.strftime("%Y_%m_%d_%H_%M_%S")
        self.save_path = os.path.join(log_dir, "loss_" + stamp)
        os.makedirs(self.save_path, exist_ok=True)
        self.losses = []
        self._txt = os.path.join(self.save_path, "epoch_loss.txt")
        self._svg = os.path.join(self.save_path, "epoch_loss.svg")

    def append_loss(self, loss):
        value = float(loss)
        self.losses.append(value)
        with open(self._txt, "a") as f:
            f.write(f"{value!r}\n")
        self._write_chart()

    # ---------------------------------------------------------------- chart
    def _running_mean(self, window=5):
        out, acc = [], 0.0
        for i, v in enumerate(self.losses):
            acc += v
            if i >= window:
                acc -= self.losses[i - window]
            out.append(acc / min(i + 1, window))
        return out

    def _write_chart(self, w=640, h=400, pad=40):
        ys = self.losses
        lo, hi = min(ys), max(ys)
        span = (hi - lo) or 1.0
        n = max(len(ys) - 1, 1)

        def pts(series):
            return " ".join(f"{pad + (w - 2 * pad) * i / n:.1f},"
                            f"{h - pad - (h - 2 * pad) * (v - lo) / span:.1f}"
                            for i, v in enumerate(series))
        svg = [f'<svg xmlns="http://www.w3.org/2000/svg" width="{w}" height="{h}">',
               f'<rect width="{w}" height="{h}" fill="white"/>',
               f'<line x1="{pad}" y1="{h - pad}" x2="{w - pad}" y2="{h - pad}" stroke="black"/>',
               f'<line x1="{pad}" y1="{pad}" x2="{pad}" y2="{h - pad}" stroke="black"/>',
               f'<polyline fill="none" stroke="crimson" stroke-width="2" points="{pts(ys)}"/>',
               f'<polyline fill="none" stroke="seagreen" stroke-dasharray="6 4" '
               f'stroke-width="2" points="{pts(self._running_mean())}"/>',
               f'<text x="{pad}" y="{pad - 10}" font-size="12">loss per epoch '
               f'({len(ys)} epochs, {lo:.4g} .. {hi:.4g}); dashed: 5-epoch running mean</text>',
               "</svg>"]
        with open(self._svg, "w") as f:
            f.write("\n".join(svg))
