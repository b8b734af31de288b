"""``python -m kubernetes_machine_learning_server_amd.serve [--port 80] [--host 0.0.0.0]``."""
import argparse
import sys


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=80)
    ap.add_argument("--workers", type=int, default=1)
    a = ap.parse_args()
    import uvicorn
    uvicorn.run("kubernetes_machine_learning_server_amd.serve.app:app", host=a.host, port=a.port,
                workers=a.workers, log_level="info")
    return 0


sys.exit(main())
