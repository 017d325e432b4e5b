"""Schema-tree leg alone (bench.tree_leg: pkg1.Message, 262144 records): one JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    print(json.dumps({"tree_pkg1": bench.tree_leg(torch.device("cuda", 0))}))


if __name__ == "__main__":
    main()
