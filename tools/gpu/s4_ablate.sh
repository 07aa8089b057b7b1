#!/bin/bash
# compute-only ablations of the LDS-DMA forward scan (timing-only builds)
M=$PWD/mamba-tts-project_amd/mtts
for v in nomem noexp nodpp noscal; do
  MTTS_LIB=$M/libmtts_$v.so timeout -k 10 120 python tools/scan_ab.py v2 2>&1 | grep north | sed "s/^/$v /" || exit 1
done
