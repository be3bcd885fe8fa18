#!/bin/bash
# Full local validation: build, host-sanitized native build of the C++ runtime,
# CPU test suite (GPU tests run on an MI355X via: python -m pytest tests -m gpu).
set -euo pipefail
cd "$(dirname "$0")/.."
bash scripts/build.sh
python -m pytest tests -x -q -m "not gpu"
if [ "${IGLOO_VALIDATE_SANITIZE:-0}" = "1" ]; then
  # host-side sanitizers only (no GPU ASan on this pool); builds a separate copy
  IGLOO_DEBUG=sanitize=address+undefined python -m igloo_amd._build --force
  python -m igloo_amd._build --force
fi
echo "validate: ok"
