#!/bin/bash
# Environment check (no installs: the ROCm image provides everything).
set -uo pipefail
ok=1
for t in hipcc python rocprofv3; do
  if command -v "$t" >/dev/null 2>&1 || [ -x "/opt/rocm/bin/$t" ]; then echo "found $t"; else echo "missing $t"; ok=0; fi
done
python - <<'PY' || ok=0
import importlib
for m in ("torch", "pyarrow", "numpy", "pybind11", "yaml"):
    importlib.import_module(m)
    print("python module", m, "ok")
import torch
print("torch", torch.__version__, "hip", torch.version.hip, "gpu visible:", torch.cuda.is_available())
PY
[ $ok = 1 ] && echo "setup: ok" || { echo "setup: incomplete"; exit 1; }
