for r in 1 2; do for v in base cls ug both; do echo "== $v"; timeout -k 10 60 hpc_suffix_array_amd/csrc/build/mb_$v 30 5 | grep -E "512x18 \+ seg grid 131072|net-sort|U\+scan|scan  "; done; done
