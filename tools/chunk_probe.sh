for f in 8 16 32 64 160; do timeout -k 5 100 python tools/kbench.py --config medium --fits $f --epochs 20 --precision bf16x3 --repeat 2 | grep rep | tail -1; done
for f in 4 8 16 40; do timeout -k 5 100 python tools/kbench.py --config large --fits $f --epochs 20 --precision bf16x3 --repeat 2 | grep rep | tail -1; done
