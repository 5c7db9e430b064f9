import re, sys, subprocess
src = sys.argv[1]
out = subprocess.run(["/opt/rocm/bin/hipcc","--offload-arch=gfx950","-O3","-std=c++17","-ffp-contract=off"]+sys.argv[3:]+["-c",src,"-o","/tmp/t/k.o","-save-temps=obj","-Rpass-analysis=kernel-resource-usage"],capture_output=True,text=True,cwd="/tmp/t").stderr
cur=None; rows={}
for line in out.splitlines():
    m=re.search(r"Function Name: (\S+)",line)
    if m: cur=m.group(1); rows[cur]={}; continue
    m=re.search(r"remark: .*?:\s+([A-Za-z ]+?)(?: \[bytes/lane\])?: (\S+) \[",line)
    if m and cur: rows[cur][m.group(1).strip()]=m.group(2)
    if "warning" in line or "error" in line: print(line)
for k,v in rows.items():
    if len(sys.argv)>2 and not re.search(sys.argv[2],k): continue
    print(f"{k[:80]:80s} vgpr={v.get('VGPRs')} agpr={v.get('AGPRs')} sgpr={v.get('TotalSGPRs')} scratch={v.get('ScratchSize')} occ={v.get('Occupancy [waves/SIMD]')}")
