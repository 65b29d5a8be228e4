"""Print bench.predict_fps (graphed vs eager bs1 detection) as JSON.

  python3 tools/predict_fps.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jabd-joint-attention-based-detector-for-small-face-detection_amd")]
import torch  # noqa: E402
import bench  # noqa: E402

if __name__ == "__main__":
    print(json.dumps(bench.predict_fps(torch.device("cuda")), indent=1))
