cd $GRAFT_REPO_ROOT && timeout -k 10 200 python -u tools/gemmbench.py ${GB_ARGS} 2>&1 | grep -v amdgpu.ids
