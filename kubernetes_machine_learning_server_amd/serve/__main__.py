"""``python -m kubernetes_machine_learning_server_amd.serve [--port 80] [--front native|uvicorn]``.

``--front native`` (default): C++ HTTP I/O threads (``--threads``) in front of the FastAPI app,
GPU matching in-process.  ``--front uvicorn``: the pure FastAPI/uvicorn stack, ``--workers``
processes.
"""
import argparse
import os
import sys


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=80)
    ap.add_argument("--front", choices=("native", "uvicorn"),
                    default=os.environ.get("SERVE_FRONT", "native"))
    ap.add_argument("--threads", type=int, default=int(os.environ.get("SERVE_THREADS", "4")),
                    help="native front: I/O threads")
    ap.add_argument("--workers", type=int, default=1, help="uvicorn front: worker processes")
    ap.add_argument("--log-level", default="info")
    a = ap.parse_args()
    if a.front == "native":
        from .front import run_native
        return run_native(a.host, a.port, a.threads)
    from .runner import run
    return run(a.host, a.port, a.workers, a.log_level)


sys.exit(main())
