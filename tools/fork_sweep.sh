# Slot-count / tail-threshold sweep with ray-tree forking (shard probe).
# usage: bash tools/fork_sweep.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-sweep}
mkdir -p gpurun_out
O=gpurun_out/fsweep_$TAG.txt
: > $O
run() {  # env... (NS: shard counts)
  echo "== $* N=$NS" >> $O
  env "$@" timeout -k 10 200 python -u tools/shard_probe.py $NS 2>/dev/null | grep '"n"' >> $O || { tail -5 $O; exit 1; }
}
NS="1 2 4 8" run RTX_X=0
NS="1 2" run RTX_TAIL=400000
NS="1 2" run RTX_TAIL=800000
NS="1" run RTX_TAIL=1600000
NS="8" run RTX_TAIL=300000
cat $O
