# cmd: bash tools/f1_pmc.sh
