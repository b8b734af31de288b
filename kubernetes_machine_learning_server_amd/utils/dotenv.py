"""Minimal ``.env`` loader (python-dotenv is not installed in this image).

Same contract as ``dotenv.load_dotenv()`` as the reference uses it
(``machine-learning/main.py:17``, ``rest_api/app/main.py:31``): read ``KEY=VALUE`` lines from
``./.env`` (or a given path) and set them only if the variable is not already in the
environment.  Supports comments, ``export`` prefixes and single/double quoted values.
"""
from __future__ import annotations

import os
import pathlib
from typing import Dict, Optional


def parse_dotenv(text: str) -> Dict[str, str]:
    out: Dict[str, str] = {}
    for raw in text.splitlines():
        line = raw.strip()
        if not line or line.startswith("#"):
            continue
        if line.startswith("export "):
            line = line[len("export "):].lstrip()
        if "=" not in line:
            continue
        key, val = line.split("=", 1)
        key, val = key.strip(), val.strip()
        if len(val) >= 2 and val[0] == val[-1] and val[0] in "\"'":
            val = val[1:-1]
        elif " #" in val:
            val = val.split(" #", 1)[0].rstrip()
        if key:
            out[key] = val
    return out


def load_dotenv(path: Optional[str] = None, override: bool = False) -> bool:
    p = pathlib.Path(path) if path else pathlib.Path.cwd() / ".env"
    if not p.is_file():
        return False
    for k, v in parse_dotenv(p.read_text(encoding="utf-8")).items():
        if override or k not in os.environ:
            os.environ[k] = v
    return True
