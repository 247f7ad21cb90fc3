cd $GRAFT_REPO_ROOT
./tools/build/bedgen 1000000 42 > /tmp/a.bed; ./tools/build/bedgen 1000000 43 > /tmp/b.bed
BEDGPU_STATS=1 ./bedops_amd/bin/bedops -i /tmp/a.bed /tmp/b.bed > /tmp/o.bed; echo rc=$?; wc -l /tmp/o.bed
