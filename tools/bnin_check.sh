# stride-1 BN-on-load: training parity tests + C4 step A/B
set -e
mkdir -p gpurun_out/bnin
timeout -k 10 600 python -u -m pytest tests/test_train.py tests/test_train_size.py tests/test_modules.py tests/test_beca_model.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/bnin/t.log 2>&1
for i in 1 2; do
JABD_DW_BNIN_S1=0 timeout -k 10 200 python3 tools/train_steps.py --kind mnv3 --steps 12 > gpurun_out/bnin/off_$i.log 2>&1
timeout -k 10 200 python3 tools/train_steps.py --kind mnv3 --steps 12 > gpurun_out/bnin/on_$i.log 2>&1
done
