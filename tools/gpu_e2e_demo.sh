#!/bin/bash
# End-to-end demo on one GPU: train the yaml ViT-tiny on the synthetic flower pool
# (cold pixelation task, then the Gaussian DDIM task), then sample from the trained
# checkpoints with the reference-compatible CLIs (cold de-pixelation sequence +
# draft->drawing img2img; DDIM k=20 samples).  Logs and PNGs -> gpurun_out/e2e/.
# EPOCHS (default 24) epochs of 16,384 images; tools/e2e_summary.py turns each
# training log into summary_*.md (steady vs end-to-end rate, epoch-boundary cost).
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
O=gpurun_out/e2e; rm -rf $O /tmp/e2e; mkdir -p $O /tmp/e2e
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; tail -${TAILN:-2} $O/$name.log | cut -c1-400
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; }
sed -e "s/epoch : \[0,2\]/epoch : [0,${EPOCHS:-24}]/" -e 's/synthetic_size : 2048/synthetic_size : 16384/' \
    -e 's/log_every : 20/log_every : 200/' configs/synthetic_tiny.yaml > /tmp/e2e/cold.yaml
sed -e "s/epoch : \[0,2\]/epoch : [0,${EPOCHS:-24}]/" -e 's/synthetic_size : 2048/synthetic_size : 16384/' \
    -e 's/log_every : 20/log_every : 200/' -e "s/framework : 'vit_tiny_synthetic'/framework : 'vit_tiny_gauss'/" \
    configs/synthetic_tiny.yaml > /tmp/e2e/gauss.yaml
echo "dataset : 'gaussian'" >> /tmp/e2e/gauss.yaml
run train_cold 600 python multi_gpu_trainer.py /tmp/e2e/cold.yaml --root /tmp/e2e
cp /tmp/e2e/Saved_Models/coldvit_tiny_synthetic/train.log $O/train_cold.log
python tools/e2e_summary.py $O/train_cold.log "cold task, ${EPOCHS:-24} epochs" > $O/summary_cold.md
run train_gauss 600 python multi_gpu_trainer.py /tmp/e2e/gauss.yaml --root /tmp/e2e
cp /tmp/e2e/Saved_Models/gaussvit_tiny_gauss/train.log $O/train_gauss.log
python tools/e2e_summary.py $O/train_gauss.log "Gaussian DDIM task, ${EPOCHS:-24} epochs" > $O/summary_gauss.md
run d2d 300 python ViT_draft2drawing.py --ckpt /tmp/e2e/Saved_Models/coldvit_tiny_synthetic/bestloss.pkl --out_dir $O
run ddim 300 python ViT.py --model vit_tiny --sample_n 64 --acc_k 20 --seq_n 6 --seq_k 100 --ckpt /tmp/e2e/Saved_Models/gaussvit_tiny_gauss/bestloss.pkl --out_dir $O
ls -la $O
