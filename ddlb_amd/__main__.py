"""``python -m ddlb_amd ...`` == the CLI (``ddlb/cli/benchmark.py:main``)."""

from ddlb_amd.cli.benchmark import main

if __name__ == "__main__":
    main()
