"""Wide / big-tag schema decode leg alone (bench.wide_leg): one JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    print(json.dumps({"decode_wide": bench.wide_leg(torch.device("cuda", 0))}))
