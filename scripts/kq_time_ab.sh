export GHIP_ALLOW_ALT_LIB=1
for rep in 1 2; do for v in ${KQT_VARS:-new h1024}; do
  if [ $v = new ]; then unset GHIP_LIB; else export GHIP_LIB=$PWD/ab_libs/lib$v.so; fi
  echo "== $v"; timeout -k 10 120 python scripts/kq_time.py 2>&1 | grep "256000\|16384" || exit 1
done; done
