# front-end A/B on the GPU box's CPU share: libmi_av1dec_base.so (HEAD) against the working tree's
set -o pipefail
R=$PWD/rav1d_amd
for la in 0 ""; do
  echo "LOOKAHEAD=${la:-pipelined}"
  LOOKAHEAD=$la timeout -k 10 400 python tools/dev/fe_ab.py $R/libmi_av1dec_base.so $R/libmi_av1dec.so issue_295,issue_318,00001141,itut_t35_10bit 11 8 || exit 1
done
