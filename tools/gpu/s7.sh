#!/bin/bash
# scan forward A/B (interleaved) + compute/memory ablations (timing-only builds)
M=$PWD/mamba-tts-project_amd/mtts
timeout -k 10 200 python tools/scan_ab.py xl dpp 2>&1 | grep north || exit 1
for v in nomem nocomp noexp nodpp noscal; do
  MTTS_LIB=$M/libmtts_$v.so timeout -k 10 200 python tools/scan_ab.py xl dpp 2>&1 | grep north | sed "s/^/$v /" || exit 1
done
