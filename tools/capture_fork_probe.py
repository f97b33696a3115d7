#!/usr/bin/env python3
"""Which fork / join patterns of side streams survive hipGraph stream capture on this ROCm (plain torch
ops, none of this package): each variant captures a few elementwise kernels on streams main / A / X in
its own child process and reports the exit code (-11: segfault at capture end) and whether the replay
computed the eager result.

    python tools/capture_fork_probe.py

Variants (-> fork, <- join; main is the capture origin):
  a_only      main->A, A->X, X<-A, A<-main                    X forked from one (side) stream
  main_only   main->X twice, joined to main each time          X forked from the origin only
  two_parents main->X, main<-X, then main->A, A->X, A<-X, main<-A      X forked from main AND from A
  two_parents_mainjoin   as two_parents, and main also waits on X at the end
  via_main    main->A; main->X (forked from main, not A), A<-X, main<-A, main<-X
  via_main_nojoin        as via_main without main<-X (X joined to main only through A)
  enter_main_wait_side   main->X, main->A, then X waits on A while capturing, A<-X, main<-A, main<-X
  reenter_main_wait_side main->X, main<-X first, then as enter_main_wait_side
"""
import json
import os
import subprocess
import sys

CHILD = r'''
import faulthandler, json, sys
faulthandler.enable()
import torch
v = sys.argv[1]
dev = torch.device("cuda:0")
main = torch.cuda.Stream(dev)
A, X = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
x = torch.zeros(1 << 16, device=dev)
y = torch.zeros(1 << 16, device=dev)

def body():
    cur = torch.cuda.current_stream(dev)
    if v == "a_only":
        A.wait_stream(cur)
        with torch.cuda.stream(A):
            X.wait_stream(A)
            with torch.cuda.stream(X):
                y.add_(1)
            A.wait_stream(X)
            x.add_(y)
        cur.wait_stream(A)
    elif v in ("enter_main_wait_side", "reenter_main_wait_side"):
        if v == "reenter_main_wait_side":
            X.wait_stream(cur)
            with torch.cuda.stream(X):
                y.add_(1)
            cur.wait_stream(X)
        X.wait_stream(cur)
        A.wait_stream(cur)
        with torch.cuda.stream(A):
            x.add_(1)
            X.wait_stream(A)
            with torch.cuda.stream(X):
                y.add_(x)
            A.wait_stream(X)
            x.add_(y)
        cur.wait_stream(A)
        cur.wait_stream(X)
    elif v == "main_only":
        for _ in range(2):
            X.wait_stream(cur)
            with torch.cuda.stream(X):
                y.add_(1)
            cur.wait_stream(X)
            x.add_(y)
    else:
        if not v.startswith("via_main"):
            X.wait_stream(cur)
            with torch.cuda.stream(X):
                y.add_(1)
            cur.wait_stream(X)
        A.wait_stream(cur)
        if v.startswith("via_main"):
            X.wait_stream(cur)
        with torch.cuda.stream(A):
            if not v.startswith("via_main"):
                X.wait_stream(A)
            with torch.cuda.stream(X):
                y.add_(2)
            A.wait_stream(X)
            x.add_(y)
        cur.wait_stream(A)
        if v in ("two_parents_mainjoin", "via_main"):
            cur.wait_stream(X)

with torch.cuda.stream(main):
    body()
torch.cuda.synchronize()
want = x.clone()
x.zero_(); y.zero_()
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=main):
    body()
x.zero_(); y.zero_()
torch.cuda.synchronize()
g.replay()
torch.cuda.synchronize()
print(json.dumps({"ok": bool(torch.equal(x, want))}))
'''

VARIANTS = ("a_only", "main_only", "two_parents", "two_parents_mainjoin", "via_main", "via_main_nojoin",
            "enter_main_wait_side", "reenter_main_wait_side")

if __name__ == "__main__":
    res = {}
    for v in VARIANTS:
        r = subprocess.run([sys.executable, "-c", CHILD, v], capture_output=True, text=True, timeout=180)
        last = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else "{}"
        res[v] = {"rc": r.returncode, **json.loads(last)}
        if r.returncode:
            res[v]["where"] = [ln.strip() for ln in r.stderr.splitlines() if ln.strip().startswith("File")][:3]
        print(v, json.dumps(res[v]), flush=True)
    print(json.dumps(res))
