# front-end A/B on the GPU box's CPU share (no GPU use): base vs work recycling (rs) vs recycling
# + parallel tile merge (pm), one temporal unit at a time (LOOKAHEAD=0) and pipelined
set -o pipefail
R=$PWD/rav1d_amd
for la in 0 ""; do
  echo "LOOKAHEAD=${la:-pipelined}"
  LOOKAHEAD=$la timeout -k 10 300 python tools/dev/fe_ab.py $R/libmi_av1dec_base.so $R/libmi_av1dec_rs.so issue_295,issue_318,00001141 7 8 || exit 1
  LOOKAHEAD=$la timeout -k 10 300 python tools/dev/fe_ab.py $R/libmi_av1dec_base.so $R/libmi_av1dec_pm.so issue_295,issue_318,00001141 7 8 || exit 1
done
