# usage: bash scripts/pmc_issue_mix.sh gpurun_out/TAG_pmc_XXXX [top]: MFMA / VALU / LDS / WAIT rates per kernel family of one pmc pass (see scripts/pmc_summary.py --rate)
python scripts/pmc_summary.py $1 --top ${2:-30} --rate SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_WAIT_INST_ANY | python -c "
import sys
lines=sys.stdin.read().splitlines()
print(lines[0])
for l in lines[1:]:
    if l.startswith('counters seen'): continue
    name=l[:72].rstrip(); rest=l[72:].split()
    # calls ms GHz MFMA% TF/s ldsconf L2hit fetch write VALU LDS WAIT
    if rest and rest[0]=='calls': print(f\"{'kernel':60s} calls     ms  MFMA%  VALU%   LDS%  WAIT%\"); continue
    print(f'{name[:60]:60s} {rest[0]:>5s} {rest[1]:>6s} {rest[3]:>6s} {rest[9]:>6s} {rest[10]:>6s} {rest[11]:>6s}')
"
