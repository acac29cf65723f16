#!/bin/bash
bash "$(dirname "$0")/gpu_prof.sh" resnet50_r1d --skip-gpt 1 --resnet-steps 10
