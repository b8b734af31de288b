"""roctx range wrapper: off by default, on with KMLS_ROCTX=1 when the ROCm roctx
library is present; push/pop must be safe without a profiler attached."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SNIPPET = """
from kubernetes_machine_learning_server_amd.ops import native
from kubernetes_machine_learning_server_amd.utils.phase_timer import PhaseTimer
m = native.load()
m.roctx_push("kmls.test"); m.roctx_pop()
t = PhaseTimer()
with t.phase("p"):
    pass
print("ENABLED" if m.roctx_enabled() else "DISABLED")
"""


def _run(env_extra):
    env = dict(os.environ, PYTHONPATH=ROOT, **env_extra)
    env.pop("KMLS_ROCTX", None) if not env_extra else None
    r = subprocess.run([sys.executable, "-c", SNIPPET], capture_output=True, text=True, env=env,
                       cwd=ROOT, timeout=120)
    assert r.returncode == 0, r.stderr
    return r.stdout.strip().splitlines()[-1]


def test_roctx_off_by_default():
    assert _run({}) == "DISABLED"


def test_roctx_on_when_requested():
    lib_present = any(os.path.exists(os.path.join("/opt/rocm/lib", n))
                      for n in ("librocprofiler-sdk-roctx.so.1", "libroctx64.so.4"))
    assert _run({"KMLS_ROCTX": "1"}) == ("ENABLED" if lib_present else "DISABLED")
