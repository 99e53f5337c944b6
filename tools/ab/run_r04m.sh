# r04m: PMC of the symbol kernels with the in-tree build — count pass + c8 hand-off, the
# emitter (sym_emit_kernel), zw_count / zw_emit, zf_count / sym_image_kernel (5 passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
CHILD=tools/sym_pmc_child.py PMC_GROUPS=tools/pmc_groups_sym.txt OUTDIR=pmc_r04m_sym timeout -k 10 900 bash tools/gpu_pmc_child.sh > gpurun_out/r04m_pmc_sym.log 2>&1 || { tail -20 gpurun_out/r04m_pmc_sym.log; exit 1; }
echo pmc done
