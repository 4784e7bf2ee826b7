#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r03s}
for dbg in 0 1 2 3; do
  echo "== VAMPOMI_WRITER_DBG=$dbg"
  VAMPOMI_WRITER_DBG=$dbg timeout -k 10 200 python -u tools/write_cost.py /tmp nowrite,write,write2 2>&1 | grep -v amdgpu.ids
done
