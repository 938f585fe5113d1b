set -o pipefail
O=gpurun_out/r05i
mkdir -p $O
export TMPDIR=/tmp
OUT=r05i/kq VARS="base=base new=new kqnochk=kqnochk kqprev=kqprev aold=aold" REPS=2 bash scripts/kqm_ab.sh || exit 1
OUT=r05i/q4 LIBS="base aold new" REPS=2 bash scripts/lib_abn.sh
