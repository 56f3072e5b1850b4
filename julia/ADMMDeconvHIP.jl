# ADMMDeconvHIP.jl -- the Julia-side binding a maintainer of georgegrosu1/admm-deconv would add so
# that the existing Flux layers (src/layers/deconv_admm.jl:215-225) and nets (src/nets/net_build.jl)
# run the MI355X-native solve.  It adds a `tvd_fft` method for ROCm device arrays next to the
# reference's CPU/CUDA methods (src/ops/ops.jl:181-188) and forwards to the C ABI in
# include/admm_deconv.h through `ccall`.  AMDGPU.jl is used ONLY for device arrays and the stream
# handle (no kernels are written in its DSL).
#
# STATUS: source only, unverified -- Julia is installed neither in the build container nor on the
# GPU box (SURVEY.md s8c), so this file has never been run.  The same C ABI is exercised from
# Python (admm-deconv_amd/admm_deconv/ops.py) by every GPU test.
module ADMMDeconvHIP

using AMDGPU
import ChainRulesCore

const LIB = normpath(joinpath(@__DIR__, "..", "admm-deconv_amd", "libadmm_deconv.so"))

const _ws = Ref{Union{Nothing, ROCArray{UInt8, 1}}}(nothing)

function _workspace(nbytes::Integer)
    w = _ws[]
    if w === nothing || length(w) < nbytes + 256
        w = ROCArray{UInt8}(undef, nbytes + 256)
        _ws[] = w
    end
    p = UInt(pointer(w))
    off = (256 - p % 256) % 256
    return Ptr{Cvoid}(p + off), Csize_t(length(w) - off)
end

_err() = unsafe_string(ccall((:admm_last_error, LIB), Cstring, ()))

"""
    tvd_fft(y::ROCArray{Float32,4}, λ, ρ=[1f0], h=ROCArray{Float32}(undef,0), isotropic=false, maxit=100)

Drop-in for `tvd_fft` (src/ops/ops.jl:181) on MI355X: same arguments, same (M,N,P,B) layout,
returns a new array.  λ and ρ are 1-element arrays (or scalars), already clamped by the layer.
"""
function tvd_fft(y::ROCArray{Float32, 4}, λ, ρ = Float32[1], h = ROCArray{Float32}(undef, 0),
                 isotropic::Bool = false, maxit::Integer = 100)
    M, N, P, B = size(y)
    kh, kw = isempty(h) ? (0, 0) : (size(h, 1), size(h, 2))
    hdev = isempty(h) ? C_NULL : pointer(h isa ROCArray ? h : ROCArray(Float32.(h)))
    lam = Float32(Array(λ)[1])     # the reference's F1-F3 hold Float64 λ/ρ (deconv_admm.jl:49,102)
    rho = Float32(Array(ρ)[1])
    nbytes = Ref{Csize_t}(0)
    rc = ccall((:admm_tvd_workspace_bytes, LIB), Cint,
               (Cint, Cint, Cint, Cint, Cint, Cint, Cint, Ref{Csize_t}), M, N, P, B, kh, kw, isotropic, nbytes)
    rc == 0 || error("admm_tvd_workspace_bytes: ", _err())
    ws, wslen = _workspace(nbytes[])
    x = similar(y)
    stream = AMDGPU.stream().stream          # hipStream_t of the task-local stream
    rc = ccall((:admm_tvd_forward_f32, LIB), Cint,
               (Ptr{Float32}, Ptr{Float32}, Cint, Cint, Cint, Cint, Ptr{Float32}, Cint, Cint, Cfloat, Cfloat,
                Cint, Cint, Ptr{Cvoid}, Csize_t, Ptr{Cvoid}),
               pointer(y), pointer(x), M, N, P, B, hdev, kh, kw, lam, rho, isotropic, maxit, ws, wslen, stream)
    rc == 0 || error("admm_tvd_forward_f32: ", _err())
    return x
end

# Zygote must not trace into the C call: the rule's pullback is the HIP adjoint through all `maxit`
# unrolled iterations -- what Zygote computes for the reference by unrolling the loop (src/train.jl:51).
# The rule's forward records the trajectory (admm_tvd_forward_record_f32) into a workspace owned by
# the pullback closure; the pullback runs only the reverse sweep (admm_tvd_backward_recorded_f32).
# Memory per call: about 8 B/px per iteration (c5: ~4.8 GB per layer), sized for MI355X's 288 GB.

# a tangent shaped like the 1-element λ / ρ the layer passes (Vector or ROCArray)
_like(a::ROCArray, v) = ROCArray(fill(eltype(a)(v), size(a)))
_like(a::AbstractArray, v) = fill(eltype(a)(v), size(a))
_like(::Number, v) = v

const _BwdSig = (Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Ptr{Float32},
                 Cint, Cint, Cint, Cint, Ptr{Float32}, Cint, Cint, Cfloat, Cfloat, Cint, Cint,
                 Ptr{Float32}, Ptr{Cvoid}, Csize_t, Ptr{Cvoid}, Ptr{Cvoid})

function ChainRulesCore.rrule(::typeof(tvd_fft), y::ROCArray{Float32, 4}, λ, ρ, h, isotropic, maxit)
    M, N, P, B = size(y)
    want_h = !isempty(h)
    kh, kw = want_h ? (size(h, 1), size(h, 2)) : (0, 0)
    hd = want_h ? (h isa ROCArray ? h : ROCArray(Float32.(h))) : nothing
    lam, rho = Float32(Array(λ)[1]), Float32(Array(ρ)[1])
    nbytes = Ref{Csize_t}(0)
    rc = ccall((:admm_tvd_backward_workspace_bytes, LIB), Cint,
               (Cint, Cint, Cint, Cint, Cint, Cint, Cint, Cint, Cint, Ref{Csize_t}),
               M, N, P, B, kh, kw, isotropic, maxit, want_h, nbytes)
    rc == 0 || error("admm_tvd_backward_workspace_bytes: ", _err())
    rec = ROCArray{UInt8}(undef, nbytes[] + 256)          # the recording; lives in the closure
    p = UInt(pointer(rec))
    off = (256 - p % 256) % 256
    ws, wslen = Ptr{Cvoid}(p + off), Csize_t(length(rec) - off)
    x = similar(y)
    rc = ccall((:admm_tvd_forward_record_f32, LIB), Cint,
               (Ptr{Float32}, Ptr{Float32}, Cint, Cint, Cint, Cint, Ptr{Float32}, Cint, Cint, Cfloat, Cfloat,
                Cint, Cint, Cint, Ptr{Cvoid}, Csize_t, Ptr{Cvoid}, Ptr{Cvoid}),
               pointer(y), pointer(x), M, N, P, B, want_h ? pointer(hd) : C_NULL, kh, kw, lam, rho,
               isotropic, maxit, want_h, ws, wslen, AMDGPU.stream().stream, C_NULL)
    rc == 0 || error("admm_tvd_forward_record_f32: ", _err())
    function tvd_fft_pullback(x̄)
        xb = ROCArray{Float32}(ChainRulesCore.unthunk(x̄))
        ȳ = similar(y)
        h̄ = want_h ? similar(hd) : nothing
        scal = AMDGPU.zeros(Float32, 2)                  # (λ̄, ρ̄)
        rc = ccall((:admm_tvd_backward_recorded_f32, LIB), Cint, _BwdSig,
                   pointer(y), pointer(xb), pointer(ȳ), want_h ? pointer(h̄) : C_NULL, pointer(scal),
                   pointer(scal) + 4, M, N, P, B, want_h ? pointer(hd) : C_NULL, kh, kw, lam, rho,
                   isotropic, maxit, pointer(x), ws, wslen, AMDGPU.stream().stream, C_NULL)
        rc == 0 || error("admm_tvd_backward_recorded_f32: ", _err())
        GC.@preserve rec nothing
        s = Array(scal)
        h̄t = want_h ? reshape(h̄, size(h)) : ChainRulesCore.NoTangent()
        return (ChainRulesCore.NoTangent(), ȳ, _like(λ, s[1]), _like(ρ, s[2]), h̄t,
                ChainRulesCore.NoTangent(), ChainRulesCore.NoTangent())
    end
    return x, tvd_fft_pullback
end

end # module

# Wiring into the reference (one line each, in the maintainer's tree):
#   src/ops/ops.jl        : include("../../julia/ADMMDeconvHIP.jl"); using .ADMMDeconvHIP
#                           tvd_fft(y::ROCArray, λ, ρ, h, iso, maxit) = ADMMDeconvHIP.tvd_fft(y, λ, ρ, h, iso, maxit)
#   src/train.jl:117-121  : `|> gpu` with Flux's AMDGPU backend (Flux.gpu_backend!("AMDGPU")) moves
#                           model and batches to ROCArrays, so (d::Admm)(x) reaches the method above.
