"""Times bench.augment_bench alone (the §8f rank 2 augmentation leg)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (puts the package on sys.path)
import torch  # noqa: E402

print(json.dumps(bench.augment_bench(torch.device("cuda:0"))))
