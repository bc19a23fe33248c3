export WC_NO_BUILD=1
for a in "--config c4 --kind payload --headers --fused" "--config c3 --len 1500 --stride 2048 --offset 14 --ragged --kind payload --headers --fused"; do
  echo "== $a"
  for rep in 1 2; do
    echo -n "prev "; WC_LIB=tools/libwccksum_prev.so timeout -k 10 120 python tools/tune.py $a --rounds 4 --iters 20 2>&1 | grep -v "round\|amdgpu"
    echo -n "new  "; timeout -k 10 120 python tools/tune.py $a --rounds 4 --iters 20 2>&1 | grep -v "round\|amdgpu"
  done
done
