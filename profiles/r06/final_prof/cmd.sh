#!/bin/bash
bash tools/final_prof.sh
