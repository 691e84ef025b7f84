# AriadneHIP.jl -- the reference-side binding of libnkhip.so (include/nkhip.h) for Ariadne.jl.
#
# UNTESTED: the build image has no Julia toolchain (SURVEY.md §8c).  This file is the `ccall` shim
# a maintainer would add so that Ariadne's own `newton_krylov!` (src/Ariadne.jl:288-372) runs its
# hot path on an MI355X without modification: device vectors (`HipVector`), the Krylov.jl vector
# primitives (the overload points examples/halovector.jl:51-147 demonstrates), the Jacobian
# operator `mul!` (src/Ariadne.jl:48-57) and, optionally, the whole device-resident GMRES/CG.
# The Python host mirror (newtonkrylov.jl_amd/ariadne_hip) binds the same symbols with ctypes and
# is what the test-suite exercises.
module AriadneHIP

using Ariadne, Krylov, LinearAlgebra, SparseArrays
import LinearAlgebra: mul!, norm, Adjoint, Transpose
import Krylov: kdot, knorm, kscal!, kaxpy!, kaxpby!, kcopy!, kfill!, kdivcopy!, kref!

const libnkhip = joinpath(@__DIR__, "..", "lib", "libnkhip.so")

const NK_BRATU1D, NK_BRATU2D, NK_HEAT2D_EULER, NK_HEAT3D_EULER = Int32(1), Int32(2), Int32(3), Int32(4)
const NK_HEAT2D_MIDPOINT, NK_HEAT3D_MIDPOINT, NK_HEAT2D_TRAPEZOID, NK_HEAT3D_TRAPEZOID = Int32(5), Int32(6), Int32(7), Int32(8)
const NK_BC_ZERO, NK_BC_PERIODIC = Int32(0), Int32(1)
const NK_USER1D, NK_USER2D, NK_USER3D = Int32(16), Int32(17), Int32(18)
const NK_JV_EXACT, NK_JV_FD = Int32(0), Int32(1)

check(rc, ctx, what) = rc == 0 || error("$what failed ($rc): " *
                                        unsafe_string(ccall((:nk_last_error, libnkhip), Cstring, (Ptr{Cvoid},), ctx.ptr)))

# --------------------------------------------------------------------------- context
mutable struct HipContext
    ptr::Ptr{Cvoid}
    function HipContext(device::Integer = 0)
        r = Ref{Ptr{Cvoid}}(C_NULL)
        rc = ccall((:nk_ctx_create, libnkhip), Cint, (Cint, Ref{Ptr{Cvoid}}), device, r)
        rc == 0 || error("nk_ctx_create($device) failed: no usable GPU (there is no CPU fallback)")
        ctx = new(r[])
        finalizer(c -> ccall((:nk_ctx_destroy, libnkhip), Cint, (Ptr{Cvoid},), c.ptr), ctx)
    end
end

"""What a context's distributed path runs (nk_dist_path, nkhip.h): transport, resident sweep, ghost
planes inside the Jv launch, ranks sharing its GPU, its PCI bus id, a sticky mailbox error."""
struct NkPathInfo
    rank::Int32
    nranks::Int32
    device::Int32
    ranks_on_device::Int32
    rccl::Int32
    mailbox::Int32
    resident_sweep::Int32
    resident_blocks::Int32
    halo_in_launch::Int32
    mailbox_error::Int32
    halo_cap::Int64
    pci_bus_id::NTuple{32, UInt8}
    jv_halo_fused::Int64
    jv_halo_separate::Int64
    sweeps_resident::Int64
    mgs_passes::Int64
    jv_fd_f0r::Int64
    jv_fd_f0_read::Int64
    halo_waits::Int64
    reduce_waits::Int64
    halo_wait_us::Float64
    reduce_wait_us::Float64
end
function path_info(ctx::HipContext)
    r = Ref{NkPathInfo}()
    check(ccall((:nk_dist_path, libnkhip), Cint, (Ptr{Cvoid}, Ref{NkPathInfo}), ctx.ptr, r), ctx, "nk_dist_path")
    p = r[]
    (rank = p.rank, nranks = p.nranks, device = p.device, ranks_on_device = p.ranks_on_device, rccl = p.rccl != 0,
     mailbox = p.mailbox != 0, resident_sweep = p.resident_sweep != 0, resident_blocks = p.resident_blocks,
     halo_in_launch = p.halo_in_launch != 0, mailbox_error = p.mailbox_error != 0, halo_cap = p.halo_cap,
     pci_bus_id = String(UInt8[c for c in p.pci_bus_id if c != 0x00]), jv_halo_fused = p.jv_halo_fused,
     jv_halo_separate = p.jv_halo_separate, sweeps_resident = p.sweeps_resident, mgs_passes = p.mgs_passes,
     jv_fd_f0r = p.jv_fd_f0r, jv_fd_f0_read = p.jv_fd_f0_read, halo_waits = p.halo_waits,
     reduce_waits = p.reduce_waits, halo_wait_us = p.halo_wait_us, reduce_wait_us = p.reduce_wait_us)
end

"""3D blocks instead of z-slabs (nk_dist_grid): px × py × pz ranks, rank = (iz py + iy) px + ix.  Call after
the ranks are connected and before allocating any vector (each 3D vector then carries x / y ghost faces)."""
process_grid!(ctx::HipContext, px::Integer, py::Integer, pz::Integer) =
    check(ccall((:nk_dist_grid, libnkhip), Cint, (Ptr{Cvoid}, Int32, Int32, Int32), ctx.ptr, px, py, pz), ctx,
          "nk_dist_grid")

# --------------------------------------------------------------------------- nk_problem (C layout)
struct NkProblem
    kind::Int32
    bc::Int32
    nx::Int64
    ny::Int64
    nz::Int64
    hx::Float64
    hy::Float64
    hz::Float64
    lambda::Float64
    a::Float64
    dt::Float64
    un::Ptr{Float64}
    user::Ptr{Cvoid}   # nk_user_ops* (NK_USER1D/2D/3D)
    alpha::Float64     # G_Midpoint!'s α (implicit.jl:17)
end
geometry(grid::NTuple{3, Int}) = NkProblem(grid[3] > 1 ? NK_HEAT3D_EULER : (grid[2] > 1 ? NK_BRATU2D : NK_BRATU1D),
                                            0, grid..., 1.0, 1.0, 1.0, 0.0, 0.0, 0.0, Ptr{Float64}(1), C_NULL, 0.5)

# --------------------------------------------------------------------------- HipVector (device HaloVector)
"""Grid function in HBM: interior x-fastest (the column-major order of a Julia array), one ghost
plane on each side of the slowest axis (zero = Dirichlet boundary; filled by the halo exchange
when distributed).  `length` is the interior count, like HaloVector (halovector.jl:17-26)."""
mutable struct HipVector <: AbstractVector{Float64}
    ctx::HipContext
    ptr::Ptr{Float64}
    grid::NTuple{3, Int}
    gen::Int     # a stamp from the process-wide counter GEN, renewed by every write this shim makes (touch!)
    f0of::Any    # set by a built-in residual F!(res, u, p): (u, u.gen, p) it was evaluated at; `nothing` once rewritten
    function HipVector(ctx::HipContext, grid::NTuple{3, Int})
        r = Ref{Ptr{Float64}}(C_NULL)
        p = geometry(grid)
        check(ccall((:nk_vec_alloc, libnkhip), Cint, (Ptr{Cvoid}, Ref{NkProblem}, Ref{Ptr{Float64}}), ctx.ptr, p, r),
              ctx, "nk_vec_alloc")
        v = new(ctx, r[], grid, next_gen(), nothing)
        finalizer(x -> ccall((:nk_vec_free, libnkhip), Cint, (Ptr{Cvoid}, Ptr{Float64}), x.ctx.ptr, x.ptr), v)
    end
    # non-owning view of library-owned storage (e.g. the Krylov workspace's x)
    HipVector(ctx::HipContext, ptr::Ptr{Float64}, grid::NTuple{3, Int}) = new(ctx, ptr, grid, next_gen(), nothing)
end
# One monotonically increasing counter for every vector and every write: a (objectid, gen) stamp can
# never repeat, even when a collected vector's objectid is reused by a new one (whose gen is fresh).
const GEN = Threads.Atomic{Int}(0)
next_gen() = Threads.atomic_add!(GEN, 1) + 1
touch!(v::HipVector) = (v.gen = next_gen(); v.f0of = nothing; v)
# the state a residual was evaluated at: u and every device vector in p (u_n of the heat problems) by
# identity and write generation, the scalars by value
stampof(x::HipVector) = (objectid(x), x.gen)
stampof(x::Tuple) = map(stampof, x)
stampof(x) = x
f0stamp(u::HipVector, p) = (stampof(u), stampof(p))
Base.size(v::HipVector) = (prod(v.grid),)
Base.similar(v::HipVector) = HipVector(v.ctx, v.grid)          # zero-filled, ghosts included
Base.zero(v::HipVector) = HipVector(v.ctx, v.grid)
Base.copy(v::HipVector) = (w = similar(v); kcopy!(length(v), w, v); w)
Base.getindex(::HipVector, ::Int) = error("scalar indexing of a HipVector; copy it to the host with Array(v)")
function Base.Array(v::HipVector)
    a = Array{Float64}(undef, v.grid)
    check(ccall((:nk_memcpy_d2h, libnkhip), Cint, (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Int64),
                v.ctx.ptr, a, v.ptr, length(v)), v.ctx, "nk_memcpy_d2h")
    return a
end
function HipVector(ctx::HipContext, a::AbstractArray{Float64})
    grid = (size(a, 1), size(a, 2), size(a, 3))
    v = HipVector(ctx, grid)
    b = Array(a)
    check(ccall((:nk_memcpy_h2d, libnkhip), Cint, (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Int64),
                ctx.ptr, v.ptr, b, length(b)), ctx, "nk_memcpy_h2d")
    return v
end

# `u .-= s .* d` (src/Ariadne.jl:344) -> one axpy kernel
function Base.Broadcast.materialize!(u::HipVector, bc::Base.Broadcast.Broadcasted)
    if bc.f === (-) && bc.args[1] === u && bc.args[2] isa Base.Broadcast.Broadcasted && bc.args[2].f === (*)
        s, d = bc.args[2].args
        return kaxpy!(length(u), -Float64(s), d::HipVector, u)  # (kaxpy! touches u)
    end
    error("unsupported broadcast on HipVector: $(bc.f)")
end
norm(v::HipVector) = knorm(length(v), v)

# --------------------------------------------------------------------------- Krylov vector primitives
const VP = Ptr{Cvoid}
function kdot(n::Integer, x::HipVector, y::HipVector)
    r = Ref{Float64}()
    check(ccall((:nk_dot, libnkhip), Cint, (VP, Int64, Ptr{Float64}, Ptr{Float64}, Ref{Float64}), x.ctx.ptr, n, x.ptr, y.ptr, r),
          x.ctx, "kdot")
    return r[]
end
function knorm(n::Integer, x::HipVector)
    r = Ref{Float64}()
    check(ccall((:nk_norm, libnkhip), Cint, (VP, Int64, Ptr{Float64}, Ref{Float64}), x.ctx.ptr, n, x.ptr, r), x.ctx, "knorm")
    return r[]
end
kscal!(n::Integer, s::Float64, x::HipVector) =
    (check(ccall((:nk_scal, libnkhip), Cint, (VP, Int64, Float64, Ptr{Float64}), x.ctx.ptr, n, s, x.ptr), x.ctx, "kscal!"); touch!(x))
kaxpy!(n::Integer, s::Float64, x::HipVector, y::HipVector) =
    (check(ccall((:nk_axpy, libnkhip), Cint, (VP, Int64, Float64, Ptr{Float64}, Ptr{Float64}), y.ctx.ptr, n, s, x.ptr, y.ptr),
           y.ctx, "kaxpy!"); touch!(y))
kaxpby!(n::Integer, s::Float64, x::HipVector, t::Float64, y::HipVector) =
    (check(ccall((:nk_axpby, libnkhip), Cint, (VP, Int64, Float64, Ptr{Float64}, Float64, Ptr{Float64}),
                 y.ctx.ptr, n, s, x.ptr, t, y.ptr), y.ctx, "kaxpby!"); touch!(y))
kcopy!(n::Integer, y::HipVector, x::HipVector) =
    (check(ccall((:nk_copy, libnkhip), Cint, (VP, Int64, Ptr{Float64}, Ptr{Float64}), y.ctx.ptr, n, y.ptr, x.ptr), y.ctx, "kcopy!"); touch!(y))
kfill!(x::HipVector, v::Float64) =
    (check(ccall((:nk_fill, libnkhip), Cint, (VP, Int64, Ptr{Float64}, Float64), x.ctx.ptr, length(x), x.ptr, v), x.ctx, "kfill!"); touch!(x))
kdivcopy!(n::Integer, y::HipVector, x::HipVector, s::Float64) =
    (check(ccall((:nk_divcopy, libnkhip), Cint, (VP, Int64, Ptr{Float64}, Ptr{Float64}, Float64), y.ctx.ptr, n, y.ptr, x.ptr, s),
           y.ctx, "kdivcopy!"); touch!(y))
kref!(n::Integer, x::HipVector, y::HipVector, c::Float64, s::Float64) =
    (check(ccall((:nk_ref, libnkhip), Cint, (VP, Int64, Ptr{Float64}, Ptr{Float64}, Float64, Float64),
                 x.ctx.ptr, n, x.ptr, y.ptr, c, s), x.ctx, "kref!"); (touch!(x), touch!(y)))

# --------------------------------------------------------------------------- residuals (F!) and mul!
"""A residual `F!(res, u, p)` with a hand-written HIP stencil (same `p` tuples as the examples).
`jv` picks the operator behind `mul!`: NK_JV_EXACT (Enzyme parity, default) or NK_JV_FD (the
north-star FD quotient); `α` is G_Midpoint!'s keyword (implicit.jl:17, default 0.5)."""
struct HipResidual{K}
    jv::Int32
    α::Float64
end
HipResidual{K}(; jv::Integer = NK_JV_EXACT, α::Real = 0.5) where {K} = HipResidual{K}(Int32(jv), Float64(α))
const bratu! = HipResidual{:bratu1d}()        # examples/bratu.jl:14-24, p = (Δx, λ)
const bratu2d! = HipResidual{:bratu2d}()      # p = (Δx, Δy, λ)
# G ∘ diffusion! (implicit.jl:8-37 ∘ heat_2D.jl:45-62), p = (uₙ, Δt, du, (a, Δx, Δy, bc!), t); 3D: (a, Δx, Δy, Δz, bc!)
const heat2d_euler! = HipResidual{:heat2d}()
const heat2d_midpoint! = HipResidual{:heat2d_midpoint}()    # α = 0.5; HipResidual{:heat2d_midpoint}(α = 0.3)
const heat2d_trapezoid! = HipResidual{:heat2d_trapezoid}()
const heat3d_euler! = HipResidual{:heat3d}()
const heat3d_midpoint! = HipResidual{:heat3d_midpoint}()
const heat3d_trapezoid! = HipResidual{:heat3d_trapezoid}()

# bc_zero! / bc_periodic! of examples/heat_2D.jl:15-38, recognised by name
bccode(bc) = nameof(bc) === :bc_periodic! ? NK_BC_PERIODIC : NK_BC_ZERO
const HEAT_KINDS = (heat2d = NK_HEAT2D_EULER, heat2d_midpoint = NK_HEAT2D_MIDPOINT, heat2d_trapezoid = NK_HEAT2D_TRAPEZOID,
                    heat3d = NK_HEAT3D_EULER, heat3d_midpoint = NK_HEAT3D_MIDPOINT, heat3d_trapezoid = NK_HEAT3D_TRAPEZOID)

problem(F::HipResidual{:bratu1d}, u::HipVector, (dx, λ)) = NkProblem(NK_BRATU1D, 0, u.grid..., dx, 1, 1, λ, 0, 0, C_NULL, C_NULL, F.α)
problem(F::HipResidual{:bratu2d}, u::HipVector, (dx, dy, λ)) = NkProblem(NK_BRATU2D, 0, u.grid..., dx, dy, 1, λ, 0, 0, C_NULL, C_NULL, F.α)
function problem(F::HipResidual{K}, u::HipVector, (un, Δt, _, fp, _t)) where {K}
    kind = HEAT_KINDS[K]
    three = kind in (NK_HEAT3D_EULER, NK_HEAT3D_MIDPOINT, NK_HEAT3D_TRAPEZOID)
    (three ? length(fp) == 5 : length(fp) == 4) || error("$(K): p[4] must be (a, Δx, Δy$(three ? ", Δz" : ""), bc!)")
    a, dx, dy = fp[1], fp[2], fp[3]
    dz = three ? fp[4] : 1.0
    return NkProblem(kind, bccode(fp[end]), u.grid..., dx, dy, dz, 0, a, Δt, un.ptr, C_NULL, F.α)
end

# --------------------------------------------------------------------------- user residuals (NK_USER*)
# Any F!(res, u, p) the caller evaluates on the device (e.g. an AMDGPU.jl / KernelAbstractions
# kernel like examples/bratu_ka.jl) -- launched on the library's stream, nk_ctx_stream(ctx).  The
# library runs the FD quotient, the GMRES basis normalisation and every reduction around it.
struct NkUserOps
    F::Ptr{Cvoid}
    J::Ptr{Cvoid}
    JT::Ptr{Cvoid}
    data::Ptr{Cvoid}
end
struct HipUserResidual{F, J}
    f!::F            # f!(res::HipVector, u::HipVector, p)
    jvp!::J          # jvp!(out, u, v, p) (exact tangent) or nothing: then only NK_JV_FD
    jv::Int32
end
HipUserResidual(f!; jvp! = nothing) = HipUserResidual(f!, jvp!, jvp! === nothing ? NK_JV_FD : NK_JV_EXACT)
libstream(ctx::HipContext) = ccall((:nk_ctx_stream, libnkhip), Ptr{Cvoid}, (Ptr{Cvoid},), ctx.ptr)

const _live = IdDict{Any, Any}()   # keeps the @cfunction closures rooted while the library may call them
function problem(F::HipUserResidual, u::HipVector, p)
    view(ptr) = HipVector(u.ctx, Ptr{Float64}(ptr), u.grid)     # non-owning
    fF = (_d, _c, res, x) -> (try F.f!(view(res), view(x), p); Cint(0) catch; Cint(1) end)
    cF = @cfunction($fF, Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}))
    cJ = F.jvp! === nothing ? nothing :
         @cfunction($((_d, _c, out, x, v) -> (try F.jvp!(view(out), view(x), view(v), p); Cint(0) catch; Cint(1) end)),
                    Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}))
    ops = Ref(NkUserOps(Base.unsafe_convert(Ptr{Cvoid}, cF),
                        cJ === nothing ? C_NULL : Base.unsafe_convert(Ptr{Cvoid}, cJ), C_NULL, C_NULL))
    _live[F] = (cF, cJ, ops, p)
    kind = u.grid[3] > 1 ? NK_USER3D : (u.grid[2] > 1 ? NK_USER2D : NK_USER1D)
    return NkProblem(kind, 0, u.grid..., 1, 1, 1, 0, 0, 0, C_NULL, Base.unsafe_convert(Ptr{Cvoid}, ops), 0.5)
end
function (F::HipUserResidual)(res::HipVector, u::HipVector, p)
    check(ccall((:nk_residual, libnkhip), Cint, (VP, Ref{NkProblem}, Ptr{Float64}, Ptr{Float64}),
                u.ctx.ptr, problem(F, u, p), res.ptr, u.ptr), u.ctx, "F!")
    touch!(res)
    return nothing
end
const AnyHipResidual = Union{HipResidual, HipUserResidual}

function (F::HipResidual)(res::HipVector, u::HipVector, p)
    check(ccall((:nk_residual, libnkhip), Cint, (VP, Ref{NkProblem}, Ptr{Float64}, Ptr{Float64}),
                u.ctx.ptr, problem(F, u, p), res.ptr, u.ptr), u.ctx, "F!")
    touch!(res).f0of = f0stamp(u, p)  # res holds F(u, p) exactly as the device residual kernel computes it
    return nothing
end

# mul!(out, J, v): more specific than Ariadne's Enzyme method (src/Ariadne.jl:48) by dispatch
const HipJacobian = Ariadne.JacobianOperator{<:AnyHipResidual, <:HipVector}
const HipJacobianT = Union{Adjoint{<:Any, <:HipJacobian}, Transpose{<:Any, <:HipJacobian}}
jvmode(J) = J.f.jv  # NK_JV_EXACT or NK_JV_FD (HipResidual and HipUserResidual both carry it)
function mul!(out::HipVector, J::HipJacobian, v::HipVector)
    F0 = jvmode(J) == NK_JV_FD ? J.res.ptr : Ptr{Float64}(C_NULL)
    check(ccall((:nk_jv, libnkhip), Cint, (VP, Ref{NkProblem}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Int32, Float64),
                out.ctx.ptr, problem(J.f, J.u, J.p), out.ptr, J.u.ptr, v.ptr, F0, jvmode(J), 0.0), out.ctx, "mul!")
    touch!(out)
    return nothing
end

# mul!(out, transpose(J), v) / adjoint (src/Ariadne.jl:87-107, Enzyme reverse mode): J(u)ᵀ v
function mul!(out::HipVector, J′::HipJacobianT, v::HipVector)
    J = parent(J′)
    check(ccall((:nk_jtv, libnkhip), Cint, (VP, Ref{NkProblem}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
                out.ctx.ptr, problem(J.f, J.u, J.p), out.ptr, J.u.ptr, v.ptr), out.ctx, "mul!(out, Jᵀ, v)")
    touch!(out)
    return nothing
end

"""k grid functions as the columns of an n × k matrix: the `Out` / `V` of the batched
mul!(Out::AbstractMatrix, J, V) (src/Ariadne.jl:67-84, :109-138)."""
struct HipMatrix <: AbstractMatrix{Float64}
    cols::Vector{HipVector}
end
HipMatrix(ctx::HipContext, grid::NTuple{3, Int}, k::Integer) = HipMatrix([HipVector(ctx, grid) for _ in 1:k])
Base.size(M::HipMatrix) = (length(first(M.cols)), length(M.cols))
Base.getindex(::HipMatrix, ::Int, ::Int) = error("scalar indexing of a HipMatrix; copy a column with Array(M.cols[j])")
colptrs(M::HipMatrix) = [c.ptr for c in M.cols]

# one fused launch per 8 columns: u, F(u) read once for all of them (nk_jv_batched)
function mul!(Out::HipMatrix, J::HipJacobian, V::HipMatrix)
    @assert size(Out, 2) == size(V, 2)
    F0 = jvmode(J) == NK_JV_FD ? J.res.ptr : Ptr{Float64}(C_NULL)
    o, v = colptrs(Out), colptrs(V)
    GC.@preserve Out V o v begin
        check(ccall((:nk_jv_batched, libnkhip), Cint,
                    (VP, Ref{NkProblem}, Int32, Ptr{Ptr{Float64}}, Ptr{Float64}, Ptr{Ptr{Float64}}, Ptr{Float64}, Int32, Float64),
                    J.u.ctx.ptr, problem(J.f, J.u, J.p), length(o), o, J.u.ptr, v, F0, jvmode(J), 0.0), J.u.ctx, "mul!(Out, J, V)")
    end
    foreach(touch!, Out.cols)
    return nothing
end
function mul!(Out::HipMatrix, J′::HipJacobianT, V::HipMatrix)
    J = parent(J′)
    @assert size(Out, 2) == size(V, 2)
    o, v = colptrs(Out), colptrs(V)
    GC.@preserve Out V o v begin
        check(ccall((:nk_jtv_batched, libnkhip), Cint,
                    (VP, Ref{NkProblem}, Int32, Ptr{Ptr{Float64}}, Ptr{Float64}, Ptr{Ptr{Float64}}),
                    J.u.ctx.ptr, problem(J.f, J.u, J.p), length(o), o, J.u.ptr, v), J.u.ctx, "mul!(Out, Jᵀ, V)")
    end
    foreach(touch!, Out.cols)
    return nothing
end

# collect(J) (src/Ariadne.jl:140-162): the exact Jacobian as a SparseMatrixCSC, assembled on the device
function Base.collect(JOp::Union{HipJacobian, HipJacobianT})
    J = JOp isa HipJacobian ? JOp : parent(JOp)
    n = length(J.u)
    dim = J.u.grid[3] > 1 ? 3 : (J.u.grid[2] > 1 ? 2 : 1)
    cap = J.f isa HipUserResidual ? min(n * n, 64 * n) : (2 * dim + 1) * n
    colptr = Vector{Int64}(undef, n + 1)
    nnz = Ref{Int64}(0)
    for attempt in 1:2
        rowval = Vector{Int64}(undef, cap)
        nzval = Vector{Float64}(undef, cap)
        rc = ccall((:nk_jacobian_collect, libnkhip), Cint,
                   (VP, Ref{NkProblem}, Ptr{Float64}, Int32, Ptr{Int64}, Ptr{Int64}, Ptr{Float64}, Int64, Ref{Int64}),
                   J.u.ctx.ptr, problem(J.f, J.u, J.p), J.u.ptr, JOp isa HipJacobian ? 0 : 1, colptr, rowval, nzval, cap, nnz)
        if rc == -2 && nnz[] > cap && attempt == 1
            cap = nnz[]
            continue
        end
        check(rc, J.u.ctx, "collect(J)")
        m = nnz[]
        return SparseMatrixCSC(n, n, colptr .+ 1, rowval[1:m] .+ 1, nzval[1:m])
    end
end

# --------------------------------------------------------------------------- optional: device-resident Krylov solve
# With only the definitions above, Krylov.jl's own gmres! runs on HipVectors: one ccall per
# primitive, a host sync per kdot/knorm.  The workspace below moves the whole Arnoldi loop into
# libnkhip.so (fused MGS passes, one sync per Arnoldi step); Ariadne reaches it through
# `krylov_workspace(algo, KrylovConstructor(res))` and `krylov_solve!` unchanged.
mutable struct HipStats      # Ariadne reads workspace.stats.niter (src/Ariadne.jl:363,367)
    niter::Int
    solved::Bool
end

mutable struct HipKrylovWorkspace
    ptr::Ptr{Cvoid}
    ctx::HipContext
    x::HipVector
    stats::HipStats
end

struct NkKrylovOpts
    restart::Int32
    reorthogonalization::Int32
    itmax::Int32
    jv_mode::Int32
    atol::Float64
    rtol::Float64
    b_norm::Float64   # 0: computed by the solve (Krylov.jl semantics)
    u_norm::Float64   # 0: computed by the solve
    u_update::Ptr{Float64}  # C_NULL: workspace.x holds the step (Ariadne applies u .-= d itself)
    N::Ptr{Cvoid}           # nk_precond* right preconditioner, C_NULL: none
    M::Ptr{Cvoid}           # nk_precond* left preconditioner, C_NULL: none
    f0_is_residual::Int32   # 1: J.res is F(J.u) as the device residual computed it (Ariadne's loop: F! just ran)
end
struct NkKrylovStats
    niter::Int64
    solved::Int32
    inconsistent::Int32
    breakdown::Int32
    status::Int32
    n_matvec::Int64
    u_norm::Float64
end

# --------------------------------------------------------------------------- preconditioners (N, M)
# Ariadne passes `N` and `M` (factories called with the step's JacobianOperator, src/Ariadne.jl:318-333)
# to krylov_solve!.  The device counterparts of examples/bratu.jl:119-157 (usable as N or as M):
#   N = hip_jacobi                           1 ./ diag(J)
#   N = hip_ilu0, krylov_kwargs = (; ldiv = true)   for  N = (J) -> ilu(collect(J))
#   N = (J) -> HipGmresPreconditioner(J, 5)  the GmresPreconditioner (algo = :fgmres)
struct NkPrecond
    kind::Int32
    diag::Ptr{Float64}
    apply::Ptr{Cvoid}
    data::Ptr{Cvoid}
    inner::Ptr{Cvoid}   # nk_workspace* (NK_PRECOND_GMRES)
    itmax::Int32
end
const NK_PRECOND_DIAG, NK_PRECOND_GMRES, NK_PRECOND_ILU0 = Int32(1), Int32(3), Int32(4)
abstract type HipPreconditioner end
struct HipDiagPreconditioner <: HipPreconditioner
    d::HipVector
    kind::Int32
end
nkprecond(P::HipDiagPreconditioner) = NkPrecond(P.kind, P.d.ptr, C_NULL, C_NULL, C_NULL, 0)
function hip_jacobi(J::Ariadne.JacobianOperator)
    d = similar(J.u)
    check(ccall((:nk_jacobian_diag, libnkhip), Cint, (VP, Ref{NkProblem}, Ptr{Float64}, Ptr{Float64}, Int32),
                J.u.ctx.ptr, problem(J.f, J.u, J.p), d.ptr, J.u.ptr, 1), J.u.ctx, "jacobi")
    return HipDiagPreconditioner(d, NK_PRECOND_DIAG)
end
function hip_ilu0(J::Ariadne.JacobianOperator)
    d = similar(J.u)
    check(ccall((:nk_ilu0_factor, libnkhip), Cint, (VP, Ref{NkProblem}, Ptr{Float64}, Ptr{Float64}),
                J.u.ctx.ptr, problem(J.f, J.u, J.p), J.u.ptr, d.ptr), J.u.ctx, "ilu0")
    return HipDiagPreconditioner(d, NK_PRECOND_ILU0)
end
struct HipGmresPreconditioner <: HipPreconditioner
    ws::Any      # HipKrylovWorkspace of the inner solve
    itmax::Int
end
HipGmresPreconditioner(J::Ariadne.JacobianOperator, itmax::Integer) =
    HipGmresPreconditioner(Krylov.krylov_workspace(:gmres, KrylovConstructor(J.res); memory = 20), itmax)
nkprecond(P::HipGmresPreconditioner) = NkPrecond(NK_PRECOND_GMRES, C_NULL, C_NULL, C_NULL, P.ws.ptr, P.itmax)

function Krylov.krylov_workspace(method::Symbol, kc::KrylovConstructor{<:HipVector}; memory::Integer = 20)
    algo = method === :gmres ? Int32(0) : method === :cg ? Int32(1) : method === :fgmres ? Int32(2) :
           error("HIP path implements :gmres, :fgmres and :cg")
    res = kc.vm
    r = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:nk_workspace_create, libnkhip), Cint, (VP, Int32, Ref{NkProblem}, Int32, Ref{Ptr{Cvoid}}),
                res.ctx.ptr, algo, geometry(res.grid), memory, r), res.ctx, "krylov_workspace")
    xptr = ccall((:nk_workspace_x, libnkhip), Ptr{Float64}, (Ptr{Cvoid},), r[])
    x = HipVector(res.ctx, xptr, res.grid)  # non-owning view (defined below)
    ws = HipKrylovWorkspace(r[], res.ctx, x, HipStats(0, false))
    finalizer(w -> ccall((:nk_workspace_destroy, libnkhip), Cint, (Ptr{Cvoid},), w.ptr), ws)
    return ws
end

function Krylov.krylov_solve!(ws::HipKrylovWorkspace, J::HipJacobian, b::HipVector;
                              restart::Bool = false, reorthogonalization::Bool = false, itmax::Integer = 0,
                              atol::Real = sqrt(eps(Float64)), rtol::Real = sqrt(eps(Float64)),
                              M = nothing, N = nothing, ldiv::Bool = false, kwargs...)
    # Ariadne forwards N = N(J) and M = M(J) when the caller gives them (src/Ariadne.jl:323-329): the
    # device GMRES / FGMRES applies both (right N, left M); the device CG takes M only
    isempty(kwargs) || error("AriadneHIP: unsupported Krylov keyword(s) $(join(keys(kwargs), ", "))")
    for P in (N, M)
        P === nothing || P isa HipPreconditioner ||
            error("AriadneHIP: preconditioners are device objects (hip_jacobi, hip_ilu0, HipGmresPreconditioner)")
        ldiv && P !== nothing && !(P isa HipDiagPreconditioner && P.kind == NK_PRECOND_ILU0) &&
            error("ldiv = true: the HIP path takes factorisations (hip_ilu0) for N and M")
    end
    nullprec = NkPrecond(0, C_NULL, C_NULL, C_NULL, C_NULL, 0)
    Nc = Ref(N === nothing ? nullprec : nkprecond(N))
    Mc = Ref(M === nothing ? nullprec : nkprecond(M))
    st = Ref{NkKrylovStats}()
    hl = Ref{Int64}(0)
    F0 = jvmode(J) == NK_JV_FD ? J.res.ptr : Ptr{Float64}(C_NULL)
    GC.@preserve Nc N Mc M begin   # the raw nk_precond* (and what they point to) stay rooted through the call
        Np = N === nothing ? Ptr{Cvoid}(C_NULL) : Ptr{Cvoid}(Base.unsafe_convert(Ptr{NkPrecond}, Nc))
        Mp = M === nothing ? Ptr{Cvoid}(C_NULL) : Ptr{Cvoid}(Base.unsafe_convert(Ptr{NkPrecond}, Mc))
        # The FD stencils may recompute F(u) from the u rows they load instead of reading J.res -- only when
        # J.res provably IS that: written by the built-in residual at this very u and p, untouched since
        # (Ariadne's loop: F!(res, u, p) just ran).  A J whose res was rewritten, or whose u / u_n changed
        # after F!, reads J.res as the FD operator's F0 (src/Ariadne.jl:48-57 semantics, mul!'s result)
        f0r = J.f isa HipResidual && J.res.f0of !== nothing && J.res.f0of == f0stamp(J.u, J.p)
        opts = NkKrylovOpts(restart, reorthogonalization, itmax, jvmode(J), atol, rtol, 0.0, 0.0, C_NULL, Np, Mp,
                            Int32(f0r ? 1 : 0))
        check(ccall((:nk_krylov_solve, libnkhip), Cint,
                    (Ptr{Cvoid}, Ref{NkProblem}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ref{NkKrylovOpts}, Ref{NkKrylovStats},
                     Ptr{Float64}, Int64, Ref{Int64}),
                    ws.ptr, problem(J.f, J.u, J.p), J.u.ptr, F0, b.ptr, opts, st, C_NULL, 0, hl), ws.ctx, "krylov_solve!")
    end
    touch!(ws.x)
    ws.stats.niter = st[].niter
    ws.stats.solved = st[].solved != 0
    return ws
end

end # module
