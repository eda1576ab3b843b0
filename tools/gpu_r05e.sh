# round 5: FPN commute / FPN kernel masks re-measured with the round-5 kernels (bench A/B)
set -u
export TMPDIR=/tmp
bash tools/ab_env.sh SFA_FPN_COMMUTE=7,SFA_FPN_COMMUTE=6,SFA_FPN_COMMUTE=4,SFA_FPN_COMMUTE=0 || exit 1
echo done
