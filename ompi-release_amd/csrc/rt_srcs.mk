# the engine sources, shared by Makefile and Makefile.san
RT_SRCS := rt/rt_core.cpp rt/op_kernels.hip rt/coll_kernels.hip rt/coll_sched.cpp rt/coll_comm.cpp \
           rt/coll_ctl.cpp rt/coll_dmabuf.cpp rt/coll_rcache.cpp rt/coll_staged.cpp rt/coll_ll_host.cpp \
           rt/coll_svc_host.cpp rt/coll_selftest.cpp rt/coll_pipe_host.cpp rt/coll_tokens.cpp rt/coll_decide.cpp \
           rt/coll_flows.cpp rt/coll_gfold.cpp \
           rt/ddt.cpp rt/ddt_kernels.hip rt/coll_ll.hip rt/coll_rules.cpp rt/p2p.cpp rt/coll_move.cpp \
           rt/coll_pipe.hip rt/coll_svc.hip rt/svc_queue.cpp
