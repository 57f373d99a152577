; optimized device IR of the fused k_seg_combine (hipcc -O3 --cuda-device-only -emit-llvm): the mode switch, the
; fallback block's own implicitarg.ptr() and the join phi -- the IR defines the pointer on both paths
  tail call void @llvm.amdgcn.s.barrier()
  fence syncscope("workgroup") acquire
  switch i32 %105, label %4466 [
    i32 3, label %123
    i32 1, label %119
  ]

119:                                              ; preds = %118
  %120 = and i32 %15, 63
  %121 = tail call ptr addrspace(4) @llvm.amdgcn.implicitarg.ptr()
  %122 = zext i32 %107 to i64
  br label %1162

...
  %330 = tail call ptr addrspace(4) @llvm.amdgcn.implicitarg.ptr()
  %331 = load i32, ptr addrspace(4) %330, align 4, !tbaa !12, !noalias !211
...
1310:  %1164 = phi ptr addrspace(4) [ %121, %119 ], [ %330, %1161 ]
1311-  %1165 = phi i32 [ %120, %119 ], [ %239, %1161 ]
1312-  %1166 = phi i1 [ false, %119 ], [ true, %1161 ]
