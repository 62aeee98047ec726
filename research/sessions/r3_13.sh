# cs2 hipGraph replay crash: capture note-only cores of both ranks and symbolize every thread's RIP
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3_13
mkdir -p $O
CFG='[["col/coll_pipeline/memcpy/cs2/graph", "col", {"algorithm": "coll_pipeline", "backend": "ipc", "s": 2, "copy_streams": 2, "graph": true}]]'
echo "core: soft $(ulimit -c) hard $(ulimit -Hc) pattern $(cat /proc/sys/kernel/core_pattern)"
PORT=29671
for r in 0 1; do
  mkdir -p /tmp/cores_r$r
  ( cd /tmp/cores_r$r && echo 0 > /proc/self/coredump_filter && \
    RANK=$r LOCAL_RANK=$r WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
    DDLB_PG_BACKEND=gloo DDLB_ALLOW_SHARED_GPU=1 DDLB_TEST_PROGRESS=1 DDLB_GRAPH_CS2=1 DDLB_GRAPH_DEBUG=1 \
    DDLB_TEST_CFGS="$CFG" PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 100 python3 -u $GRAFT_REPO_ROOT/tests/_ipc_worker.py > $O/rank$r.log 2>&1 ) &
done
wait
for r in 0 1; do
  echo "== rank $r"; tail -80 $O/rank$r.log
  ls -la /tmp/cores_r$r
  for c in /tmp/cores_r$r/core*; do [ -f "$c" ] && python3 scripts/core_notes.py "$c" > $O/core_rank$r.txt 2>&1; done
  [ -f $O/core_rank$r.txt ] && cat $O/core_rank$r.txt | head -60
done
exit 0
