#!/bin/bash
# Build the native extension (C++ SQL frontend + gfx950 HIP kernels) in-tree and check it imports.
set -euo pipefail
cd "$(dirname "$0")/.."
python -m igloo_amd._build "$@"
python -c "import igloo_amd, igloo_amd.ops._lib as L; L.native(); print('igloo_amd', igloo_amd.__version__, 'native ok')"
