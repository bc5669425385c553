#!/bin/bash
# BiLSTM layer time vs workgroup count, at 4, 8 and 16 sequences per workgroup
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
for ns in 4 8 16; do
  ND_LSTM_SEQ=$ns timeout -k 10 120 python -u tools/lstm_sweep.py > $O/lstm_sweep_$ns.log 2>&1 || exit $?
  cat $O/lstm_sweep_$ns.log
done
