#!/bin/bash
set -o pipefail
bash tools/quick32.sh && bash tools/run_stamps.sh
