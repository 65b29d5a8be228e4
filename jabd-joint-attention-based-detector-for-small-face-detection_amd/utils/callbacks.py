"""Per-epoch loss log for the training scripts' `LossHistory(log_dir)` /
`.append_loss(value)` calls (reference interface: utils/callbacks.py:7-49,
called at e.g. train_50_3_r.py:276,350).

Host bookkeeping only, out of the hot path.  As the
reference: each run gets its own directory `log_dir/loss_<stamp>` (creating
it fails if it exists, :17), and every appended value goes to
`epoch_loss_<stamp>.txt` as `str(loss)` one per line (:21-23).  The chart is a
small dependency-free SVG, `epoch_loss_<stamp>.svg`, with a running mean,
where the reference draws `epoch_loss_<stamp>.png` with matplotlib and a
Savitzky-Golay smoothing (:26-46): matplotlib is not a dependency here.
"""
import os
import time


class LossHistory:
    def __init__(self, log_dir):
        self.log_dir = log_dir
        self.time_str = time.strftime("%Y_%m_%d_%H_%M_%S")
        self.save_path = os.path.join(log_dir, "loss_" + self.time_str)
        self.losses = []
        os.makedirs(self.save_path)
        self._txt = os.path.join(self.save_path, "epoch_loss_" + self.time_str + ".txt")
        self._svg = os.path.join(self.save_path, "epoch_loss_" + self.time_str + ".svg")

    def append_loss(self, loss):
        self.losses.append(loss)
        with open(self._txt, "a") as f:
            f.write(str(loss))
            f.write("\n")
        self._write_chart()

    # ---------------------------------------------------------------- chart
    def _running_mean(self, window=5):
        out, acc = [], 0.0
        vals = [float(v) for v in self.losses]
        for i, v in enumerate(vals):
            acc += v
            if i >= window:
                acc -= vals[i - window]
            out.append(acc / min(i + 1, window))
        return out

    def _write_chart(self, w=640, h=400, pad=40):
        ys = [float(v) for v in self.losses]
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
