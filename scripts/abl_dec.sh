set -u
cd scripts/micro
for b in dec_abl_0 dec_stamp enc_abl_0; do
  timeout -k 10 60 ./$b || exit 1
done
