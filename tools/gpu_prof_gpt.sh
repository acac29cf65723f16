#!/bin/bash
# rocprofv3 of the current GPT-3 13B bench step (1 warmup + 2 timed steps).
bash "$(dirname "$0")/gpu_prof.sh" gpt13b_r1e --steps 2 --warmup 1 --resnet 0
