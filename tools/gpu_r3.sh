#!/bin/bash
# Round-3 GPU session: new parity tests, the --gpus 2 rehearsal, FFT-domain decoder A/B.
# usage (on the GPU box via gpurun): bash tools/gpu_r3.sh <step...>
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 \
        --timeout-method thread -m gpu \
        -k "fftdec or runtime_kernels or decode_cache or all_parity or threads or repair or filler or large_verify or verify_batch or fillers" \
        > gpurun_out/t_r3.log 2>&1 || exit 1 ;;
    gpus2)
      CESS_DIST_BACKEND=gloo CESS_DEVICE=0 timeout -k 10 300 python -u bench.py --gpus 2 \
        --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/b_gpus2.json 2> gpurun_out/b_gpus2.err \
        || exit 1 ;;
    c6)
      for e in ${FD_E:-5 8 16 32}; do
        for f in 0 5; do
          timeout -k 10 120 python -u bench.py --config 6 --erasures $e --fftdec-min $f --steps 50 \
            --warmup 5 --no-cpu-baseline >> gpurun_out/c6_ab.jsonl 2>> gpurun_out/c6_ab.err || exit 1
        done
      done ;;
    fdtests)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 \
        --timeout-method thread -m gpu -k "fftdec or decode_cache or all_parity or reconstruct or dispatch" \
        > gpurun_out/t_fd.log 2>&1 || exit 1 ;;
    fdab)  # k_fftdec_m on each library of FD_LIBS (CESS_EC_LIB), k_rthx beside
      for e in ${FD_E:-5 8 16 32}; do
        for lib in ${FD_LIBS:-cess_amd/libcessec.so}; do
          CESS_EC_LIB=$PWD/$lib timeout -k 10 120 python -u bench.py --config 6 --erasures $e \
            --fftdec-mode 1 --steps 50 --warmup 5 --no-cpu-baseline >> gpurun_out/fd_ab.jsonl \
            2>> gpurun_out/fd_ab.err || exit 1
        done
        timeout -k 10 120 python -u bench.py --config 6 --erasures $e --fftdec-min ${FD_RTHX:-0} --steps 50 \
          --warmup 5 --no-cpu-baseline >> gpurun_out/fd_ab.jsonl 2>> gpurun_out/fd_ab.err || exit 1
      done ;;
    fddtests)  # the formal-derivative decoder against the C oracle (and the dispatch)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 \
        --timeout-method thread -m gpu -k "fftdec" > gpurun_out/t_fdd.log 2>&1 || exit 1 ;;
    fddab)  # k_fftdec_d (mode 2) beside k_fftdec_m (mode 1) and the default pick, per erasure count
      for e in ${FD_E:-8 16 24 32}; do
        for md in 2 1 0; do
          timeout -k 10 120 python -u bench.py --config 6 --erasures $e --fftdec-mode $md --steps 50 \
            --warmup 5 --no-cpu-baseline >> gpurun_out/fdd_ab.jsonl 2>> gpurun_out/fdd_ab.err || exit 1
        done
      done ;;
    fddlibs)  # k_fftdec_d builds of FD_LIBS (CESS_EC_LIB) against each other, interleaved
      for rep in 1 2; do
        for e in ${FD_E:-8 32}; do
          for lib in ${FD_LIBS:-cess_amd/libcessec.so}; do
            CESS_EC_LIB=$PWD/$lib timeout -k 10 120 python -u bench.py --config 6 --erasures $e \
              --fftdec-mode 2 --steps 50 --warmup 5 --no-cpu-baseline | sed "s|^{|{\"lib\": \"$lib\", |" \
              >> gpurun_out/fdd_libs.jsonl 2>> gpurun_out/fdd_libs.err || exit 1
          done
        done
      done ;;
  esac
done
