#!/usr/bin/env python3
"""JSON-config entry point (parity: ``scripts/run_benchmark.py``).

    python scripts/run_benchmark.py                      # scripts/config.json
    python scripts/run_benchmark.py path/to/config.json
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 scripts/run_benchmark.py cfg.json
"""

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(os.path.abspath(__file__)), "config.json")
    try:
        with open(path) as f:
            config = json.load(f)
    except (OSError, json.JSONDecodeError) as e:
        print(f"Error loading config file {path}: {e}")
        sys.exit(1)
    from ddlb_amd.cli import run_benchmark

    run_benchmark(config)


if __name__ == "__main__":
    main()
