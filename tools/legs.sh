# Source me: LEGS0 = bench.py flags that turn every side leg off (combine with the one leg wanted).
LEGS0="--cpu-seconds 0 --host-steps 0 --packetize-reps 0 --proxy-reps 0 --reassembly-reps 0 --crypto-reps 0 --flat-reps 0 --boutique-reps 0 --payload-reps 0 --mixed-reps 0 --config3-reps 0 --trace-reps 0 --per-record 0 --ref-reps 0"
