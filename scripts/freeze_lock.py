#!/usr/bin/env python3
"""Print requirements.lock: exact versions of the runtime and test dependencies installed in
this image (the reference pins its environments with uv.lock: machine-learning/uv.lock,
rest_api/uv.lock)."""
import importlib.metadata as md
import platform

PKGS = ["numpy", "pandas", "torch", "fastapi", "starlette", "uvicorn", "jinja2", "MarkupSafe",
        "pydantic", "pydantic_core", "prometheus_client", "pytz", "pybind11", "python-dateutil",
        "tzdata", "six", "typing_extensions", "anyio", "h11", "click", "annotated_types", "idna",
        "exceptiongroup", "aiohttp", "aiosignal", "frozenlist", "multidict", "yarl", "propcache",
        "attrs", "async_timeout", "aiohappyeyeballs", "pytest", "pytest-timeout", "hypothesis",
        "httpx", "httpcore", "certifi", "sortedcontainers", "iniconfig", "pluggy", "packaging",
        "tomli", "filelock", "fsspec", "sympy", "networkx", "mpmath"]


def main() -> None:
    print("# Exact versions of every runtime / test dependency, pinned from the MI355X build image")
    print(f"# (ROCm 7.2.0, Python {platform.python_version()}, PyTorch {md.version('torch')}).")
    print("# The reference pins its environments with uv.lock (machine-learning/uv.lock,")
    print("# rest_api/uv.lock); the images install exactly these with --no-deps.")
    print("# Regenerate: python scripts/freeze_lock.py > requirements.lock")
    for p in PKGS:
        try:
            print(f"{p}=={md.version(p)}")
        except md.PackageNotFoundError:
            pass


if __name__ == "__main__":
    main()
