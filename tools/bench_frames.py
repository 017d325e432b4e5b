"""Device frame index leg alone (bench.frames_leg) on the 1M Flat16 batch: one JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    _, _, _, _, stream, ends = bench.make_batch(1 << 20, 0x5EC0DE, dev)
    print(json.dumps({"frames": bench.frames_leg(stream, ends, dev)}))


if __name__ == "__main__":
    main()
