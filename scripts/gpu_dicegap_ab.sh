for v in 0 dgrad 1; do
  PMU_WINO4=$v timeout 280 python -u -m pytest -q -s -m gpu -p no:cacheprovider tests/test_bf16_gpu.py -k dice_gap > gpurun_out/dg_$v.log 2>&1
  grep -o "C5_DICE_GAP.*" gpurun_out/dg_$v.log | cut -c 13- > gpurun_out/dg_$v.json
  python -c "
import json,sys; d=json.load(open('gpurun_out/dg_$v.json')); f=d['fp32']
print('$v', 'fp32 gap eval', [round(x,6) for x in f['dice_gap_eval']], 'train', [round(x,6) for x in f['dice_gap_train']], 'agree', f['argmax_agreement_vs_oracle_eval'], f['argmax_agreement_vs_oracle_train'])
"
done
