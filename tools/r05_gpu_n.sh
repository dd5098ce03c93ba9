#!/bin/bash
# Round 5, GPU call n: frontier bookkeeping simplification -- streams must be
# byte-identical to the previous build; gzip times A/B.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05n
mkdir -p $O
T() { timeout -k 10 "$@"; }
for r in 1 2; do
  OFL_CODEC_LIB=tools/bin/var/libofl_codec_gzbase2.so T 200 python -u tools/tlz_ab.py base >> $O/ab.jsonl 2>> $O/ab.err || exit 12
  T 200 python -u tools/tlz_ab.py new >> $O/ab.jsonl 2>> $O/ab.err || exit 13
done
echo "r05n done"
