#!/bin/bash
# (lib_exp/libpair.so is csrc/unet.hip with profiles/r6/conv_pair/k_conv3_bf16_paired_taps.diff applied, built by tools/exp_build.py --src unet pair)
# Round 6: bf16 halo conv with a 4-slot weight ring and one barrier per two taps (lib_exp/libpair.so; pairns:
# the same without the scheduling fence between an interval's taps) against the product build: bitwise
# fingerprints (tools/c3_pair_check.py), then interleaved conv_micro timings at B = 344 and the 344-tile
# bf16 U-Net forward (tools/bench_configs4.py --unet-only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${1:-gpurun_out/r6/pair}
mkdir -p $O
for v in base pair pairns; do
  if [ $v = base ]; then L=""; else L="red-diffeq_amd/lib_exp/lib$v.so"; fi
  RDQ_HIP_LIB=$L timeout -k 10 200 python -u tools/c3_pair_check.py $O/fp_$v.json > $O/fp_$v.log 2>&1 || { echo "fp $v rc=$?"; tail -5 $O/fp_$v.log; exit 1; }
done
python3 tools/c3_pair_check.py --cmp $O/fp_base.json $O/fp_pair.json; python3 tools/c3_pair_check.py --cmp $O/fp_base.json $O/fp_pairns.json
for rep in 1 2; do
  for v in base pair pairns; do
    if [ $v = base ]; then L=""; else L="red-diffeq_amd/lib_exp/lib$v.so"; fi
    RDQ_HIP_LIB=$L timeout -k 10 200 python -u tools/conv_micro.py --B 344 --bf16 --reps 10 >> $O/micro_$v.jsonl 2>> $O/micro.err || { echo "micro $v rc=$?"; exit 1; }
    RDQ_HIP_LIB=$L timeout -k 10 300 python -u tools/bench_configs4.py --unet-only --precision bf16 >> $O/unet_$v.jsonl 2>> $O/unet.err || { echo "unet $v rc=$?"; tail -5 $O/unet.err; exit 1; }
    echo "$v $rep $(tail -1 $O/unet_$v.jsonl | cut -c1-200)"
  done
done
for v in base pair pairns; do echo "== $v"; cat $O/micro_$v.jsonl; done
