#!/bin/bash
set -u
mkdir -p gpurun_out/flake
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u scripts/probe/resln_flake.py 60 > gpurun_out/flake/probe.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/flake/probe.log | grep -v " 0 bad" ; grep -c " 0 bad" gpurun_out/flake/probe.log
