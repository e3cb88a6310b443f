set -o pipefail
cd $GRAFT_REPO_ROOT
PMC_TAG=_tlds bash tools/pmc_plane.sh native table 20 ylds=2 rows_per_wave=1 || exit 1
PMC_TAG=_t64r1 bash tools/pmc_plane.sh native table 20 ylds=3 yt_rows=1 || exit 1
PMC_TAG=_t64r2 bash tools/pmc_plane.sh native table 20 ylds=3 yt_rows=2 || exit 1
