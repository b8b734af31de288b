"""``python -m kubernetes_machine_learning_server_amd.serve [--port 80] [--workers N]``."""
import argparse
import sys

from .runner import run


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=80)
    ap.add_argument("--workers", type=int, default=1)
    ap.add_argument("--log-level", default="info")
    a = ap.parse_args()
    return run(a.host, a.port, a.workers, a.log_level)


sys.exit(main())
