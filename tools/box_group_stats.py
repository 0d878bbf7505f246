# Run and group statistics of the coarse box kernel on config 2 (profiles/r02/experiments/ab_box_groups.txt):
# per (window, angle), runs of equal box corners and groups of runs whose corners fit a W x H cell
# rectangle (base = first corner - bo). Host-only numpy, seeded config-2 world and scans.
import sys, math, numpy as np
sys.path[:0]=['roborts-edu-slam_amd','oracle']
from roborts_csm import worlds
from roborts_csm.params import headline_levels
lv = headline_levels()[0]
print(lv)
w = worlds.make_world(2000,2000,0.05,seed=20261015)
b = worlds.make_scan_batch(w, 8, seed=1000)
res=w.resolution
def stats(pts, pose, base_off):
    s=1/res; cx=s*pose[0]+s*w.offset[0]; cy=s*pose[1]+s*w.offset[1]
    ns = int(round(lv.search_space_size/lv.search_space_resolution))+1
    x0 = cx - (lv.search_space_size/res)*0.5; y0 = cy - (lv.search_space_size/res)*0.5
    na = int(math.floor(2*lv.search_angle_offset/lv.search_angle_resolution))+1
    runs=groups=0
    for a in range(na):
        th = pose[2]-lv.search_angle_offset + a*lv.search_angle_resolution
        c,sn=math.cos(th),math.sin(th)
        lx=c*pts[:,0]-sn*pts[:,1]; ly=sn*pts[:,0]+c*pts[:,1]
        ix=np.trunc((lx+x0)+0.5).astype(int); iy=np.trunc((ly+y0)+0.5).astype(int)
        # runs
        corners=[(ix[0],iy[0])]
        for i in range(1,len(ix)):
            if (ix[i],iy[i])!=corners[-1]: corners.append((ix[i],iy[i]))
        runs+=len(corners)
        g=0; base=None
        for (x,y) in corners:
            if base is None or not (0<=x-base[0]<=3 and 0<=y-base[1]<=3):
                g+=1; base=(x-base_off[0], y-base_off[1])
        groups+=g
    return runs/na, groups/na
for k in range(4):
    pts=b.points_cells[b.offsets[k]:b.offsets[k+1]]
    print(k, len(pts), [stats(pts, b.init_poses[k], bo) for bo in [(0,0),(1,1),(2,2)]])
print("---- window sizes")
def stats2(pts, pose, W, H, bo):
    s=1/res; cx=s*pose[0]+s*w.offset[0]; cy=s*pose[1]+s*w.offset[1]
    x0 = cx - (lv.search_space_size/res)*0.5; y0 = cy - (lv.search_space_size/res)*0.5
    na = int(math.floor(2*lv.search_angle_offset/lv.search_angle_resolution))+1
    runs=groups=0
    for a in range(na):
        th = pose[2]-lv.search_angle_offset + a*lv.search_angle_resolution
        c,sn=math.cos(th),math.sin(th)
        lx=c*pts[:,0]-sn*pts[:,1]; ly=sn*pts[:,0]+c*pts[:,1]
        ix=np.trunc((lx+x0)+0.5).astype(int); iy=np.trunc((ly+y0)+0.5).astype(int)
        corners=[(ix[0],iy[0])]
        for i in range(1,len(ix)):
            if (ix[i],iy[i])!=corners[-1]: corners.append((ix[i],iy[i]))
        runs+=len(corners)
        g=0; base=None
        for (x,y) in corners:
            if base is None or not (0<=x-base[0]<W and 0<=y-base[1]<H):
                g+=1; base=(x-bo[0], y-bo[1])
        groups+=g
    return round(runs/na), round(groups/na)
for (W,H,bo) in [(4,4,(1,1)),(3,3,(1,1)),(4,1,(1,0)),(1,4,(0,1)),(2,2,(0,0)),(4,4,(2,1))]:
    tot_r=tot_g=0
    for k in range(8):
        pts=b.points_cells[b.offsets[k]:b.offsets[k+1]]
        r,g=stats2(pts,b.init_poses[k],W,H,bo); tot_r+=r; tot_g+=g
    print(W,H,bo,'runs',tot_r/8,'groups',tot_g/8, 'ratio %.2f'%(tot_r/tot_g))
print("---- dy-only")
for (W,H,bo) in [(1,4,(0,1)),(1,4,(0,2)),(1,4,(0,0)),(2,4,(0,1)),(2,4,(1,1))]:
    tot_r=tot_g=0
    for k in range(8):
        pts=b.points_cells[b.offsets[k]:b.offsets[k+1]]
        r,g=stats2(pts,b.init_poses[k],W,H,bo); tot_r+=r; tot_g+=g
    print(W,H,bo,'runs',tot_r/8,'groups',tot_g/8, 'ratio %.2f'%(tot_r/tot_g))
