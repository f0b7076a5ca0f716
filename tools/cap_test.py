import sys, torch
sys.path[:0] = ['super-resolution-climate_amd', '.']
d = torch.device('cuda', 0)
x = torch.ones(1 << 20, device=d)
st = torch.cuda.Stream(device=d)
evf, evj = torch.cuda.Event(), torch.cuda.Event()
def work():
    main = torch.cuda.current_stream()
    evf.record(main); st.wait_event(evf)
    x.mul_(2)
    with torch.cuda.stream(st):
        x.add_(1)
    evj.record(st); main.wait_event(evj)
work(); torch.cuda.synchronize()
g = torch.cuda.CUDAGraph(); s = torch.cuda.Stream(device=d)
s.wait_stream(torch.cuda.current_stream())
try:
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            work()
    print("torch-only fork/join capture OK")
except Exception as e:
    print("torch-only capture failed:", e)
# now with an srmi kernel on the side stream
from srmi.engine import axpy
y = torch.ones(1 << 20, device=d)
def work2():
    main = torch.cuda.current_stream()
    evf.record(main); st.wait_event(evf)
    with torch.cuda.stream(st):
        axpy(y, x, 1.0)
    evj.record(st); main.wait_event(evj)
work2(); torch.cuda.synchronize()
g2 = torch.cuda.CUDAGraph()
try:
    with torch.cuda.stream(s):
        with torch.cuda.graph(g2, stream=s):
            work2()
    print("srmi fork/join capture OK")
except Exception as e:
    print("srmi capture failed:", e)
