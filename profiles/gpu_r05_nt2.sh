#!/bin/bash
# Round 5: non-temporal sample loads in k_integrate, more interleaved pairs against the shipped build.
set -o pipefail
export TMPDIR=/tmp
bash profiles/gpu_r05_ab.sh nt2 4 real= ntld=noetic-slam_amd/lib/var/libtsdf_hip_ntld.so
