# FM chain register-operand kernels vs the LDS-staged ones (ab/libkdfm_base.so from HEAD): isolated time and
# bitwise outputs
set -o pipefail
OUT=gpurun_out/r5zk
mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 120 python3 -u tools/fmchain_micro.py 30 $OUT/new.pt > $OUT/new$i.log 2>&1 || { echo "micro failed"; tail -5 $OUT/new$i.log; exit 3; }
  grep fm_chain $OUT/new$i.log | sed 's/^/new: /'
  KDFM_LIB=ab/libkdfm_base.so timeout -k 10 120 python3 -u tools/fmchain_micro.py 30 $OUT/base.pt > $OUT/base$i.log 2>&1 || { echo "micro failed"; tail -5 $OUT/base$i.log; exit 3; }
  grep fm_chain $OUT/base$i.log | sed 's/^/base: /'
done
python3 -c "
import torch
a = torch.load('$OUT/new.pt'); b = torch.load('$OUT/base.pt')
for k in a: print(k, 'bitwise' if torch.equal(a[k], b[k]) else 'DIFF %g' % (a[k].float() - b[k].float()).abs().max())
"
rm -f $OUT/*.pt
