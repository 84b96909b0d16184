#!/bin/bash
# Round 6 GPU batch L: C3 (BiomedCLIP ViT-B/16 + PubMedBERT-256, batch 64) bench line and its two-stream
# run-to-run determinism probe, plus the C2 probe at batch 32 (the test's size) for the record.
cd "$(dirname "$0")/.."
out=gpurun_out/r06_l; mkdir -p $out
timeout -k 10 600 python3 -u bench.py --model biomedclip-vit_b16-pubmedbert256 --batch 64 --no-cpu-baseline --no-roofline > $out/bench_c3_n1_b64.json 2> $out/bench_c3.err || { tail -20 $out/bench_c3.err; exit 1; }
cut -c1-200 $out/bench_c3_n1_b64.json
timeout -k 10 600 python3 -u tools/determinism_probe.py --model biomedclip-vit_b16-pubmedbert256 --batch 64 --steps 3 --repeats 6 --variants conc --summary --self-ref > $out/determinism_c3_b64.log 2>&1 || { tail -20 $out/determinism_c3_b64.log; exit 2; }
tail -1 $out/determinism_c3_b64.log
timeout -k 10 600 python3 -u tools/determinism_probe.py --batch 32 --steps 3 --repeats 8 --variants conc --summary --self-ref > $out/determinism_c2_b32.log 2>&1 || { tail -20 $out/determinism_c2_b32.log; exit 3; }
tail -1 $out/determinism_c2_b32.log
