import sys, numpy as np
sys.path[:0]=['.', 'distributed-deep-q_amd']
import ddq
for S,B in [(16,256),(16,64),(16,65),(16,128),(128,2)]:
    net = ddq.DeepQNet(batch=B, frame=S)
    rng=np.random.default_rng(0)
    st=rng.integers(0,256,(B,4,S,S)).astype(np.float32)
    act=np.zeros((B,4,1,1),np.float32); act[:,0]=1
    try:
        net.write_minibatch(st,act,np.zeros((B,1,1,1),np.float32),st,np.ones((B,1,1,1),np.float32))
        print(S,B,net.forward_backward())
    except Exception as e:
        print(S,B,"ERR",e)
    net.close()
