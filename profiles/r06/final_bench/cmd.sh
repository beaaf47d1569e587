#!/bin/bash
bash tools/final_bench.sh
