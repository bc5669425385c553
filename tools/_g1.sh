set -u
P=tools/overlap_trace.py
bash tools/gpu.sh py ov_one256 $P --mode one --B 256 && \
bash tools/gpu.sh py ov_one128 $P --mode one --B 128 && \
bash tools/gpu.sh py ov_ser2 $P --mode serial --B 256 --parts 2 && \
bash tools/gpu.sh py ov_conc2 $P --mode conc --B 256 --parts 2 && \
bash tools/gpu.sh py ov_conc4 $P --mode conc --B 256 --parts 4 && \
bash tools/gpu.sh py ov_conc2_nog $P --mode conc --B 256 --parts 2 --graphs 0 --iters 3 && \
bash tools/gpu.sh py ov_one256_nog $P --mode one --B 256 --graphs 0 --iters 3 && \
bash tools/gpu.sh ptrace ovt_conc2 $GRAFT_REPO_ROOT/$P --mode conc --B 256 --parts 2 --iters 2 --warmup 1 && \
bash tools/gpu.sh ptrace ovt_one128 $GRAFT_REPO_ROOT/$P --mode one --B 128 --iters 2 --warmup 1
