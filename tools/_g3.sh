set -u
P=tools/overlap_trace.py
bash tools/gpu.sh py ov_ext3_768 $P --mode ext --B 768 --parts 3 && \
bash tools/gpu.sh py ov_ext2_512b $P --mode ext --B 512 --parts 2 --iters 20 && \
bash tools/gpu.sh py ov_one256b $P --mode one --B 256 --iters 20 && \
bash tools/gpu.sh py ov_nano_one256 $P --mode one --B 256 --encoder nano && \
bash tools/gpu.sh py ov_nano_ext2_512 $P --mode ext --B 512 --parts 2 --encoder nano
