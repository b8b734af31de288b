#!/usr/bin/env bash
# Build + push both images (reference: */buildAndPushToDockerhub.sh).  REGISTRY=... to override.
set -euo pipefail
REGISTRY=${REGISTRY:-kmls-amd}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
docker build -f "$ROOT/deploy/docker/Dockerfile.api" -t "$REGISTRY/api:latest" "$ROOT"
docker build -f "$ROOT/deploy/docker/Dockerfile.job" -t "$REGISTRY/job:latest" "$ROOT"
docker push "$REGISTRY/api:latest"
docker push "$REGISTRY/job:latest"
