# round 5 / 9: long-K A/B of the tile raster (DDLB_RASTER_G: m-blocks per raster group of
# tile_mn) on the BASELINE long-K shapes, bf16 and MX-fp8, against hipBLASLt in the same processes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_9
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/ab_env_gemm.py --knob DDLB_RASTER_G --values 4,2,8,16 --shapes 5,2,6 --rounds 3 > $O/ab_raster_bf16.txt 2>&1 || { echo "ab failed"; tail -20 $O/ab_raster_bf16.txt; exit 1; }
tail -16 $O/ab_raster_bf16.txt
timeout -k 10 500 python -u scripts/ab_env_gemm.py --knob DDLB_RASTER_G --values 4,2,8 --shapes 5,2 --dtype float8_e4m3fn --modes mx --rounds 3 > $O/ab_raster_mx.txt 2>&1 || { echo "ab mx failed"; tail -20 $O/ab_raster_mx.txt; exit 1; }
tail -12 $O/ab_raster_mx.txt
