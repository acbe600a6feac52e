import json,os,time,sys
sys_path_fix = __import__("sys").path.insert(0, __import__("os").getcwd())
from rav1d_amd.av1dec import stream_events
G="tests/golden/streams"; V={v["name"]:v for v in json.load(open(G+"/vectors.json"))}
for name in sys.argv[1].split(","):
    data=open(os.path.join(G,V[name]["file"]),"rb").read()
    out=[]
    for th in [1,8]:
        best=1e9
        for r in range(3):
            t=time.perf_counter(); n=sum(1 for e in stream_events(data,th)); best=min(best,time.perf_counter()-t)
        out.append(round(best*1e3,1))
    print(name, out)
