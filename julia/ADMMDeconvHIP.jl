# ADMMDeconvHIP.jl -- the Julia-side binding a maintainer of georgegrosu1/admm-deconv would add so
# that the existing Flux layers (src/layers/deconv_admm.jl:215-225) and nets (src/nets/net_build.jl)
# run the MI355X-native solve.  It adds a `tvd_fft` method for ROCm device arrays next to the
# reference's CPU/CUDA methods (src/ops/ops.jl:181-188) and forwards to the C ABI in
# include/admm_deconv.h through `ccall`.  AMDGPU.jl is used ONLY for device arrays and the stream
# handle (no kernels are written in its DSL).
#
# STATUS: source only, never executed -- Julia is installed neither in the build container nor on the
# GPU box (SURVEY.md s8c).  tests/test_julia_abi.py (CPU) checks that every `ccall` type tuple below
# matches the C prototype in include/admm_deconv.h, and tests/test_gpu_julia_abi.py (GPU) replays
# each `ccall` with the same argument tuples through ctypes (device λ/ρ pointers, `pointer(scal) + 4`
# for ρ̄, C_NULL with kh = kw = 0 for the empty PSF).
module ADMMDeconvHIP

using AMDGPU
import ChainRulesCore

const LIB = normpath(joinpath(@__DIR__, "..", "admm-deconv_amd", "libadmm_deconv.so"))

# One forward workspace per HIP stream: concurrent tasks on different streams never share scratch
# state, and work on one stream is ordered, so a stream's workspace is reused only after the work
# that used it (the rule the Python binding follows, ops.py `_default_workspace`).
const _ws = Dict{UInt, ROCArray{UInt8, 1}}()
# Temporaries handed to the library by pointer (converted PSF, λ, ρ) stay referenced here until the
# next call on the same stream, which the stream orders after the kernels that read them.
const _keep = Dict{UInt, Any}()
const _lock = ReentrantLock()

_stream() = AMDGPU.stream().stream                 # hipStream_t of the task-local stream
_key(s) = UInt(s)

function _workspace(s, nbytes::Integer)
    lock(_lock) do
        w = get(_ws, _key(s), nothing)
        if w === nothing || length(w) < nbytes + 256
            w = ROCArray{UInt8}(undef, nbytes + 256)
            _ws[_key(s)] = w
        end
        p = UInt(pointer(w))
        off = (256 - p % 256) % 256
        return w, Ptr{Cvoid}(p + off), Csize_t(length(w) - off)
    end
end

_err() = unsafe_string(ccall((:admm_last_error, LIB), Cstring, ()))

# λ / ρ as the reference passes them: 1-element device arrays (tvd_fft(y, λ::CGPUArray, ρ::CGPUArray),
# ops.jl:99,181).  A Float32 ROCArray is passed as is (read in-kernel, no host sync); anything else
# (the Float64 `zeros(1) .+ λ` of ADMMDeconvF1-F3, deconv_admm.jl:49,102,155-156; a host vector; a
# number) becomes a Float32 device copy -- an upload or a device cast, never a readback.
_dev32(a::ROCArray{Float32}) = a
_dev32(a::ROCArray) = Float32.(a)
_dev32(a::AbstractArray) = ROCArray(Float32.(vec(a)))
_dev32(a::Number) = ROCArray(Float32[a])

_psf(h) = isempty(h) ? nothing : (h isa ROCArray{Float32} ? h : ROCArray(Float32.(h)))

const _FwdSig = (Ptr{Float32}, Ptr{Float32}, Cint, Cint, Cint, Cint, Ptr{Float32}, Cint, Cint,
                 Ptr{Float32}, Ptr{Float32}, Cint, Cint, Ptr{Cvoid}, Csize_t, Ptr{Cvoid}, Ptr{Cvoid})

"""
    tvd_fft(y::ROCArray{Float32,4}, λ, ρ=[1f0], h=ROCArray{Float32}(undef,0), isotropic=false, maxit=100)

Drop-in for `tvd_fft` (src/ops/ops.jl:181) on MI355X: same arguments, same (M,N,P,B) layout,
returns a new array.  λ and ρ are 1-element arrays (or scalars), already clamped by the layer; as
device arrays they are read in-kernel (admm_tvd_forward_dev_f32), so the call never syncs the host.
"""
function tvd_fft(y::ROCArray{Float32, 4}, λ, ρ = Float32[1], h = ROCArray{Float32}(undef, 0),
                 isotropic::Bool = false, maxit::Integer = 100)
    M, N, P, B = size(y)
    hd = _psf(h)
    kh, kw = hd === nothing ? (0, 0) : (size(h, 1), size(h, 2))
    lam, rho = _dev32(λ), _dev32(ρ)
    nbytes = Ref{Csize_t}(0)
    rc = ccall((:admm_tvd_workspace_bytes, LIB), Cint,
               (Cint, Cint, Cint, Cint, Cint, Cint, Cint, Ref{Csize_t}), M, N, P, B, kh, kw, isotropic, nbytes)
    rc == 0 || error("admm_tvd_workspace_bytes: ", _err())
    s = _stream()
    w, ws, wslen = _workspace(s, nbytes[])
    x = similar(y)
    GC.@preserve y x hd lam rho w begin
        rc = ccall((:admm_tvd_forward_dev_f32, LIB), Cint, _FwdSig,
                   pointer(y), pointer(x), M, N, P, B, hd === nothing ? C_NULL : pointer(hd), kh, kw,
                   pointer(lam), pointer(rho), isotropic, maxit, ws, wslen, s, C_NULL)
    end
    rc == 0 || error("admm_tvd_forward_dev_f32: ", _err())
    lock(_lock) do
        _keep[_key(s)] = (hd, lam, rho)       # alive until the stream has run the kernels that read them
    end
    return x
end

# Zygote must not trace into the C call: the rule's pullback is the HIP adjoint through all `maxit`
# unrolled iterations -- what Zygote computes for the reference by unrolling the loop (src/train.jl:51).
# The rule's forward records the trajectory (admm_tvd_forward_record_dev_f32) into a workspace owned by
# the pullback closure; the pullback runs only the reverse sweep (admm_tvd_backward_recorded_dev_f32).
# Memory per call: about 8 B/px per iteration (c5: ~4.8 GB per layer), sized for MI355X's 288 GB.

# a tangent shaped like the 1-element λ / ρ the layer passes (device arrays stay on the device)
_like(a::ROCArray, g::ROCArray) = reshape(eltype(a).(g), size(a))
_like(a::AbstractArray, g::ROCArray) = reshape(eltype(a).(Array(g)), size(a))
_like(::Number, g::ROCArray) = Array(g)[1]

const _RecSig = (Ptr{Float32}, Ptr{Float32}, Cint, Cint, Cint, Cint, Ptr{Float32}, Cint, Cint,
                 Ptr{Float32}, Ptr{Float32}, Cint, Cint, Cint, Ptr{Cvoid}, Csize_t, Ptr{Cvoid}, Ptr{Cvoid})
const _BwdSig = (Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Ptr{Float32},
                 Cint, Cint, Cint, Cint, Ptr{Float32}, Cint, Cint, Ptr{Float32}, Ptr{Float32}, Cint, Cint,
                 Ptr{Float32}, Ptr{Cvoid}, Csize_t, Ptr{Cvoid}, Ptr{Cvoid})

function ChainRulesCore.rrule(::typeof(tvd_fft), y::ROCArray{Float32, 4}, λ, ρ, h, isotropic, maxit)
    M, N, P, B = size(y)
    hd = _psf(h)
    want_h = hd !== nothing
    kh, kw = want_h ? (size(h, 1), size(h, 2)) : (0, 0)
    lam, rho = _dev32(λ), _dev32(ρ)
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
    GC.@preserve y x hd lam rho rec begin
        rc = ccall((:admm_tvd_forward_record_dev_f32, LIB), Cint, _RecSig,
                   pointer(y), pointer(x), M, N, P, B, want_h ? pointer(hd) : C_NULL, kh, kw,
                   pointer(lam), pointer(rho), isotropic, maxit, want_h, ws, wslen, _stream(), C_NULL)
    end
    rc == 0 || error("admm_tvd_forward_record_dev_f32: ", _err())
    function tvd_fft_pullback(x̄)
        xb = ROCArray{Float32}(ChainRulesCore.unthunk(x̄))
        ȳ = similar(y)
        h̄ = want_h ? similar(hd) : nothing
        scal = AMDGPU.zeros(Float32, 2)                  # (λ̄, ρ̄), left on the device
        GC.@preserve y xb ȳ h̄ scal hd lam rho x rec begin
            rc = ccall((:admm_tvd_backward_recorded_dev_f32, LIB), Cint, _BwdSig,
                       pointer(y), pointer(xb), pointer(ȳ), want_h ? pointer(h̄) : C_NULL, pointer(scal),
                       pointer(scal) + 4, M, N, P, B, want_h ? pointer(hd) : C_NULL, kh, kw,
                       pointer(lam), pointer(rho), isotropic, maxit, pointer(x), ws, wslen, _stream(), C_NULL)
        end
        rc == 0 || error("admm_tvd_backward_recorded_dev_f32: ", _err())
        # the pullback closure captures rec, lam, rho, hd and x, and the returned tangents reference ȳ, h̄
        # and scal: all outlive the reverse sweep the stream runs before anything reads the gradients
        h̄t = want_h ? reshape(h̄, size(h)) : ChainRulesCore.NoTangent()
        return (ChainRulesCore.NoTangent(), ȳ, _like(λ, view(scal, 1:1)), _like(ρ, view(scal, 2:2)), h̄t,
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
