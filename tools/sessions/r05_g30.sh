# Round 5 (GPU box): sampe -B 5 bulk vs serial reader, HEAD binary vs the -G build, twice each
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=$(mktemp -d)
G=tests/golden
python3 - "$T" <<'PY'
import sys
recs = open("tests/golden/pe100_2.fq").read().split("\n")
k = 4 * (len(recs) // 8)
s = recs[k + 1]
recs[k + 1] = s[:40] + "\n" + s[40:]
open(sys.argv[1] + "/r2.fq", "w").write("\n".join(recs))
PY
timeout -k 10 60 ibwa_amd/bin/ibwa-amd aln -B 5 -f $T/0.sai $G/g1m $G/pe100_1.fq 2> /dev/null &&
timeout -k 10 60 ibwa_amd/bin/ibwa-amd aln -B 5 -f $T/1.sai $G/g1m $T/r2.fq 2> /dev/null || exit 1
for bin in ibwa-amd.head ibwa-amd; do
  for k in 1 2; do
    timeout -k 10 60 ibwa_amd/bin/$bin sampe -R -f $T/$bin.bulk$k.sam $G/g1m $T/0.sai $T/1.sai $G/pe100_1.fq $T/r2.fq 2> $T/$bin.bulk$k.err || exit 1
    IBWA_SAMPE_SERIAL_READ=1 timeout -k 10 60 ibwa_amd/bin/$bin sampe -R -f $T/$bin.serial$k.sam $G/g1m $T/0.sai $T/1.sai $G/pe100_1.fq $T/r2.fq 2> $T/$bin.serial$k.err || exit 1
  done
done
md5sum $T/*.sam
cp $T/*.sam $T/*.err gpurun_out/ 2>/dev/null; mkdir -p gpurun_out/g30 && mv gpurun_out/*.sam gpurun_out/*.err gpurun_out/g30/
