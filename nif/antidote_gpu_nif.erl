%% antidote_gpu_nif — Erlang side of the MI355X materialization engine.
%%
%% Drop-in for the hot path of clocksi_materializer:materialize/4
%% (src/clocksi_materializer.erl:82-101), materializer_vnode update/2 and
%% read/6 (src/materializer_vnode.erl:96-110) over an engine-owned partition
%% log, and stable_time_functions:get_min_time/1
%% (src/stable_time_functions.erl:51-85).  Terms are encoded here (per-call
%% path) or in the NIF (partition path, exact interning) into the SoA arrays
%% of include/antidote_gpu.h; the NIF (antidote_gpu_nif.c) runs the HIP
%% kernels on a dirty scheduler.  Built only where erl_nif.h exists; see
%% INTEGRATION.md for the patches that route the reference through it.
-module(antidote_gpu_nif).

-export([open/1, materialize/6, gst_min/5, select_base/7]).
-export([materialize/4, get_min_time/1]).
%% clocksi_materializer:new/1, materialize_eager/3; materializer:update_snapshot/3
-export([new/1, materialize_eager/3, update_snapshot/3]).
%% engine-owned partition (one per materializer_vnode, keys of every type)
-export([part_open/5, part_update/6, part_read/6, part_materialize/7, part_gc/3,
         part_gc_due/3, part_stats/1, part_key_meta/3, part_store/8]).
-export([new_partition/3, update/3, read/5, read_cached/5, read_from/7, gc/3]).

-on_load(init/0).

-include("antidote.hrl").

-define(COUNTER, 1).
-define(SET_AW, 2).
-define(REGISTER_MV, 3).
-define(F_NEWSS, 1).
-define(F_CT_IGNORE, 2).
-define(F_ERR_UNEXPECTED, 4).
-define(F_ERR_CORRUPTED, 8).
-define(INVALID_EFFECT, -16#8000000000000000).
-define(U64_MAX, 16#FFFFFFFFFFFFFFFF).

init() ->
    Dir = case code:priv_dir(antidote) of
              {error, _} -> filename:dirname(code:which(?MODULE));
              P -> P
          end,
    erlang:load_nif(filename:join(Dir, "antidote_gpu_nif"), 0).

open(_Device) -> erlang:nif_error(not_loaded).
materialize(_Ctx, _Type, _NDcs, _Log, _Read, _CapOff) -> erlang:nif_error(not_loaded).
gst_min(_Ctx, _NDcs, _NParts, _Clocks, _Defined) -> erlang:nif_error(not_loaded).
select_base(_Ctx, _NDcs, _CacheOff, _Clocks, _ClockMask, _R, _RMask) -> erlang:nif_error(not_loaded).
part_open(_Ctx, _Type, _NDcs, _NKeys, _Cached) -> erlang:nif_error(not_loaded).
part_update(_Part, _Key, _Type, _OcPairs, _TxId, _Effect) -> erlang:nif_error(not_loaded).
part_read(_Part, _Key, _Type, _RPairs, _TxId, _Gc) -> erlang:nif_error(not_loaded).
part_materialize(_Part, _Key, _Type, _RPairs, _Sct, _TxId, _Base) -> erlang:nif_error(not_loaded).
part_gc(_Part, _Key, _ThresholdPairs) -> erlang:nif_error(not_loaded).
part_store(_Part, _Key, _Type, _CommitTimePairs, _NewLastOp, _Count, _Value, _Gc) -> erlang:nif_error(not_loaded).
part_gc_due(_Part, _Key, _Type) -> erlang:nif_error(not_loaded).
part_stats(_Part) -> erlang:nif_error(not_loaded).
part_key_meta(_Part, _Key, _Type) -> erlang:nif_error(not_loaded).

ctx() ->
    case persistent_term:get({?MODULE, ctx}, undefined) of
        undefined ->
            {ok, C} = open(0),
            persistent_term:put({?MODULE, ctx}, C),
            C;
        C -> C
    end.

type_id(antidote_crdt_counter_pn) -> ?COUNTER;
type_id(antidote_crdt_set_aw) -> ?SET_AW;
type_id(antidote_crdt_register_mv) -> ?REGISTER_MV.

%% ---------------------------------------------------------------------------
%% clocksi_materializer:materialize/4, same arguments and results.
materialize(Type, TxId, MinSnapshotTime,
            #snapshot_get_response{snapshot_time = SCT, ops_list = Ops,
                                   materialized_snapshot = #materialized_snapshot{value = Base}}) ->
    TypeId = type_id(Type),
    OpList = oldest_first(Ops),
    Dcs = dc_table([MinSnapshotTime, SCT | [clock_of(Op) || {_, Op} <- OpList]]),
    D = max(1, length(Dcs)),
    Idx = maps:from_list(lists:zip(Dcs, lists:seq(0, length(Dcs) - 1))),
    TxCodes = txid_codes(TxId, OpList),
    {Log, Terms, Tags0, Toks0} = encode_log(Type, TypeId, OpList, Idx, D, TxCodes),
    {BaseOff, BaseTag, BaseTok, Tags, Toks} = encode_base(TypeId, Base, Tags0, Toks0),
    {Read, CapOff} = encode_read(TypeId, Idx, D, MinSnapshotTime, SCT, txid_code(TxId, TxCodes),
                                 Base, {BaseOff, BaseTag, BaseTok}, Log),
    {ok, R} = materialize(ctx(), TypeId, D, Log, Read, CapOff),
    decode(Type, TypeId, Dcs, D, R, Terms, Tags, Toks).

%% clocksi_materializer:new/1 (src/clocksi_materializer.erl:41-43) =
%% materializer:create_snapshot/1 (src/materializer.erl:45-47).
new(Type) -> Type:new().

%% clocksi_materializer:materialize_eager/3 (src/clocksi_materializer.erl:
%% 270-274) -> materializer:materialize_eager/3 (src/materializer.erl:61-70):
%% every effect applied in order, no snapshot checks, the first failure
%% returned.  Run as materialize/4 over ops whose only clock entry is one
%% synthetic DC at time 0, read at that DC's time 0, SCT = ignore: every op
%% passes the filter (oc <= R) and the fold is the eager fold.
materialize_eager(Type, Snapshot, Effects) ->
    N = length(Effects),
    Ops = [{Id, #clocksi_payload{key = eager, type = Type, op_param = E,
                                 snapshot_time = dict:new(), commit_time = {'$eager', 0},
                                 txid = ignore}}
           || {Id, E} <- lists:zip(lists:seq(N, 1, -1), lists:reverse(Effects))],
    Resp = #snapshot_get_response{snapshot_time = ignore, ops_list = Ops, number_of_ops = N,
                                  materialized_snapshot = #materialized_snapshot{last_op_id = 0,
                                                                                 value = Snapshot}},
    case materialize(Type, ignore, dict:store('$eager', 0, dict:new()), Resp) of
        {ok, Value, _NewLastOp, _LastOpCt, _IsNewSS, _Count} -> Value;
        {error, Reason} -> {error, Reason}
    end.

%% materializer:update_snapshot/3 (src/materializer.erl:51-58).
update_snapshot(Type, Snapshot, Effect) ->
    case materialize_eager(Type, Snapshot, [Effect]) of
        {error, Reason} -> {error, Reason};
        Value -> {ok, Value}
    end.

oldest_first(Ops) when is_list(Ops) -> lists:reverse(Ops);
oldest_first(Tuple) when is_tuple(Tuple) ->
    {Length, _} = element(2, Tuple),
    [element(?FIRST_OP + I, Tuple) || I <- lists:seq(0, Length - 1)].

clock_of(#clocksi_payload{snapshot_time = SS, commit_time = {Dc, Ct}}) ->
    dict:store(Dc, Ct, SS).

dc_table(Clocks) ->
    lists:usort(lists:append([dict:fetch_keys(C) || C <- Clocks, C =/= ignore])).

row(Clock, Idx, D) ->
    Vals = lists:foldl(fun({Dc, T}, A) -> setelement(maps:get(Dc, Idx) + 1, A, T) end,
                       erlang:make_tuple(D, 0), dict:to_list(Clock)),
    Mask = lists:foldl(fun(Dc, M) -> M bor (1 bsl maps:get(Dc, Idx)) end, 0, dict:fetch_keys(Clock)),
    W = (D + 63) div 64,
    {<< <<V:64/native>> || V <- tuple_to_list(Vals) >>, <<Mask:(64 * W)/little>>}.

%% TxIds are interned exactly per call (a map keyed by the term itself, =:=
%% semantics; a #tx_id{} holds integers and a pid, where == and =:= agree):
%% is_op_in_snapshot compares TxId == Op#clocksi_payload.txid
%% (src/clocksi_materializer.erl:220), so no two distinct TxIds may share a code.
txid_codes(TxId, OpList) ->
    All = [TxId | [Op#clocksi_payload.txid || {_, Op} <- OpList]],
    {Map, _} = lists:foldl(fun(ignore, Acc) -> Acc;
                              (T, {M, N}) -> case maps:is_key(T, M) of
                                                 true -> {M, N};
                                                 false -> {maps:put(T, N, M), N + 1}
                                             end
                           end, {#{}, 1}, All),
    Map.

encode_log(Type, TypeId, OpList, Idx, D, TxCodes) ->
    KeyType = case lists:all(fun({_, #clocksi_payload{type = T}}) -> T =:= Type end, OpList) of
                  true -> TypeId;
                  false -> 16#FF
              end,
    case TypeId of
        ?COUNTER ->
            N = length(OpList),
            {Rows, Masks} = lists:unzip([row(clock_of(Op), Idx, D) || {_, Op} <- OpList]),
            Ids = << <<Id:32/native>> || {Id, _} <- OpList >>,
            TxIds = << <<(txid_code(Op#clocksi_payload.txid, TxCodes)):64/native>> || {_, Op} <- OpList >>,
            Base = {<<0:64/native, N:64/native>>, <<KeyType:8>>, iolist_to_binary(Rows),
                    iolist_to_binary(Masks), Ids, TxIds},
            {Effs, Terms} = lists:foldl(
                fun({_, #clocksi_payload{op_param = E}}, {Acc, T}) when is_integer(E),
                                                                        E > ?INVALID_EFFECT,
                                                                        E < 16#8000000000000000 ->
                        {[<<E:64/signed-native>> | Acc], T};
                   ({_, #clocksi_payload{op_param = E}}, {Acc, T}) ->
                        {[<<?INVALID_EFFECT:64/signed-native>> | Acc], [{length(Acc), E} | T]}
                end, {[], []}, OpList),
            {erlang:append_element(erlang:append_element(
                 erlang:append_element(erlang:append_element(erlang:append_element(Base,
                     iolist_to_binary(lists:reverse(Effs))), <<>>), <<>>), <<>>), <<>>),
             maps:from_list(Terms), #{}, #{}};
        _ ->
            %% one entry per {Elem, Add, Rem} part (add_all / remove_all) and
            %% per extra add token, all under the op's id
            encode_tag_log(KeyType, OpList, TypeId, Idx, D, TxCodes)
    end.

txid_code(ignore, _) -> 0;
txid_code(T, Codes) -> maps:get(T, Codes).

encode_tag_log(KeyType, OpList, TypeId, Idx, D, TxCodes) ->
    %% entries: {OpId, Op, TagTerm | invalid, AddTok | none, Rems}
    Entries = lists:append([op_entries(TypeId, Id, Op) || {Id, Op} <- OpList]),
    N = length(Entries),
    {Rows, Masks} = lists:unzip([row(clock_of(Op), Idx, D) || {_, Op, _, _, _} <- Entries]),
    Ids = << <<Id:32/native>> || {Id, _, _, _, _} <- Entries >>,
    TxIds = << <<(txid_code(Op#clocksi_payload.txid, TxCodes)):64/native>> || {_, Op, _, _, _} <- Entries >>,
    {Tags, Toks, TagA, AddA, OffA, RemA, Terms, _} = lists:foldl(
        fun({_, Op, invalid, _, _}, {Tg, Tk, TagA0, AddA0, OffA0, RemA0, Tm, I}) ->
                {Tg, Tk, [<<16#FFFFFFFF:32/native>> | TagA0], [<<0:64>> | AddA0],
                 [hd(OffA0) | OffA0], RemA0, maps:put(I, Op#clocksi_payload.op_param, Tm), I + 1};
           ({_, _, TagTerm, AddTok, Rems}, {Tg, Tk, TagA0, AddA0, OffA0, RemA0, Tm, I}) ->
                {Tg1, TagId} = intern(TagTerm, Tg),
                {Tk1, AddId} = case AddTok of none -> {Tk, 0}; _ -> intern(AddTok, Tk) end,
                {Tk2, RemIds} = lists:foldl(fun(X, {T, L}) -> {T2, Id} = intern(X, T), {T2, [Id | L]} end,
                                            {Tk1, []}, Rems),
                Off = hd(OffA0) + length(RemIds),
                {Tg1, Tk2, [<<TagId:32/native>> | TagA0], [<<AddId:64/native>> | AddA0],
                 [Off | OffA0], [[<<R:64/native>> || R <- lists:reverse(RemIds)] | RemA0], Tm, I + 1}
        end, {#{}, #{}, [], [], [0], [], #{}, 0}, Entries),
    Log = {<<0:64/native, N:64/native>>, <<KeyType:8>>, iolist_to_binary(Rows),
           iolist_to_binary(Masks), Ids, TxIds, <<>>,
           iolist_to_binary(lists:reverse(TagA)), iolist_to_binary(lists:reverse(AddA)),
           << <<O:32/native>> || O <- lists:reverse(OffA) >>,
           iolist_to_binary(lists:reverse(RemA))},
    {Log, Terms, Tags, Toks}.

%% the entries of one op: set_aw parts {Elem, Adds, Rems} (several for
%% add_all / remove_all; a part with n add tokens gives n entries, the removals
%% riding on the first), register_mv {V, Tok, Ovr} / {reset, Ovr}; an effect the
%% CRDT could not apply stays one invalid entry (update/2 raises at read)
op_entries(TypeId, Id, Op = #clocksi_payload{op_param = E}) ->
    case parts(TypeId, E) of
        {ok, Parts} -> [{Id, Op, Tag, Add, Rems} || {Tag, Add, Rems} <- Parts];
        error -> [{Id, Op, invalid, none, []}]
    end.

parts(?SET_AW, Parts) when is_list(Parts) ->
    try {ok, lists:append([set_part(P) || P <- Parts])}
    catch _:_ -> error
    end;
parts(?REGISTER_MV, {reset, Ovr}) when is_list(Ovr) -> {ok, [{reset, none, Ovr}]};
parts(?REGISTER_MV, {Value, Token, Ovr}) when is_list(Ovr) -> {ok, [{Value, Token, Ovr}]};
parts(_, _) -> error.

set_part({Elem, [], Rems}) when is_list(Rems) -> [{Elem, none, Rems}];
set_part({Elem, [A | More], Rems}) when is_list(Rems), is_list(More) ->
    [{Elem, A, Rems} | [{Elem, X, []} || X <- More]].

%% #materialized_snapshot.value of a set_aw ([{Elem, [Tok]}]) or register_mv
%% ([{Value, Token}]) base, as (elem/value, token) pairs through the same
%% intern maps as the log
encode_base(?SET_AW, State, Tags, Toks) ->
    base_pairs([{E, T} || {E, Ts} <- State, T <- Ts], Tags, Toks);
encode_base(?REGISTER_MV, State, Tags, Toks) ->
    base_pairs(State, Tags, Toks);
encode_base(_, _, Tags, Toks) ->
    {<<>>, <<>>, <<>>, Tags, Toks}.

base_pairs(Pairs, Tags, Toks) ->
    {TagB, TokB, Tags1, Toks1} = lists:foldl(
        fun({E, T}, {TgA, TkA, Tg, Tk}) ->
                {Tg1, TagId} = intern(E, Tg),
                {Tk1, TokId} = intern(T, Tk),
                {[<<TagId:32/native>> | TgA], [<<TokId:64/native>> | TkA], Tg1, Tk1}
        end, {[], [], Tags, Toks}, Pairs),
    N = length(Pairs),
    {<<0:64/native, N:64/native>>, iolist_to_binary(lists:reverse(TagB)),
     iolist_to_binary(lists:reverse(TokB)), Tags1, Toks1}.

intern(Term, Map) ->
    case maps:find(Term, Map) of
        {ok, Id} -> {Map, Id};
        error -> Id = maps:size(Map) + 1, {maps:put(Term, Id, Map), Id}
    end.

encode_read(TypeId, Idx, D, R, SCT, TxCode, Base, {BaseOff, BaseTag, BaseTok}, Log) ->
    {RRow, RMask} = row(R, Idx, D),
    {SRow, SMask, SIgn} = case SCT of
                              ignore -> {<<>>, <<>>, <<1:8>>};
                              _ -> {Sr, Sm} = row(SCT, Idx, D), {Sr, Sm, <<0:8>>}
                          end,
    Tx = <<TxCode:64/native>>,
    BaseValue = case TypeId of ?COUNTER -> <<Base:64/signed-native>>; _ -> <<>> end,
    Read = {<<0:64/native>>, RRow, RMask, SRow, SMask, SIgn, Tx, BaseValue, BaseOff, BaseTag,
            BaseTok},
    Cap = case TypeId of
              ?COUNTER -> <<>>;
              _ -> N = byte_size(element(9, Log)) div 8 + byte_size(BaseTok) div 8,
                   <<0:64/native, N:64/native>>
          end,
    {Read, Cap}.

decode(Type, TypeId, Dcs, D, {Value, Hole, LastCt, LastCtMask, Count, Flags, ErrPos, OutN, OutTag, OutTok},
       Terms, Tags, Toks) ->
    <<F:32/native>> = Flags,
    <<C:32/native>> = Count,
    <<H:64/signed-native>> = Hole,
    if
        F band ?F_ERR_CORRUPTED =/= 0 -> erlang:error(corrupted_ops_cache);
        F band ?F_ERR_UNEXPECTED =/= 0 ->
            <<E:32/native>> = ErrPos,
            {error, {unexpected_operation, maps:get(E, Terms, undefined), Type}};
        true ->
            Ct = case F band ?F_CT_IGNORE of
                     0 -> decode_clock(Dcs, D, LastCt, LastCtMask);
                     _ -> ignore
                 end,
            V = case TypeId of
                    ?COUNTER -> <<X:64/signed-native>> = Value, X;
                    _ -> decode_state(TypeId, OutN, OutTag, OutTok, Tags, Toks)
                end,
            {ok, V, H, Ct, F band ?F_NEWSS =/= 0, C}
    end.

decode_clock(Dcs, D, Vals, MaskBin) ->
    W = (D + 63) div 64,
    <<Mask:(64 * W)/little>> = MaskBin,
    L = [V || <<V:64/native>> <= Vals],
    dict:from_list([{Dc, lists:nth(I + 1, L)} || {Dc, I} <- lists:zip(Dcs, lists:seq(0, length(Dcs) - 1)),
                                                 (Mask bsr I) band 1 =:= 1]).

decode_state(TypeId, <<N:32/native>>, TagBin, TokBin, Tags, Toks) ->
    RTags = maps:from_list([{I, T} || {T, I} <- maps:to_list(Tags)]),
    RToks = maps:from_list([{I, T} || {T, I} <- maps:to_list(Toks)]),
    Pairs = lists:sublist(lists:zip([T || <<T:32/native>> <= TagBin], [K || <<K:64/native>> <= TokBin]), N),
    Terms = [{maps:get(T, RTags), maps:get(K, RToks)} || {T, K} <- Pairs],
    case TypeId of
        ?SET_AW ->
            orddict:from_list(lists:foldr(fun({E, K}, Acc) ->
                                                  orddict:update(E, fun(L) -> [K | L] end, [K], Acc)
                                          end, [], Terms));
        ?REGISTER_MV -> lists:sort(Terms)
    end.

%% ---------------------------------------------------------------------------
%% stable_time_functions:get_min_time/1 on the device.
get_min_time(Dict) ->
    Entries = dict:to_list(Dict),
    Dcs = lists:usort(lists:append([dict:fetch_keys(V) || {_, V} <- Entries, V =/= undefined])),
    D = max(1, length(Dcs)),
    Rows = [case V of
                undefined -> << <<?U64_MAX:64/native>> || _ <- lists:seq(1, D) >>;
                _ -> << <<(case dict:find(Dc, V) of {ok, T} -> T; error -> ?U64_MAX end):64/native>>
                        || Dc <- Dcs >>
            end || {_, V} <- Entries],
    Defined = << <<(case V of undefined -> 0; _ -> 1 end):8>> || {_, V} <- Entries >>,
    {ok, Vec} = gst_min(ctx(), D, length(Entries), iolist_to_binary(Rows), Defined),
    Words = [W || <<W:64/native>> <= Vec],
    dict:from_list([{Dc, T} || {Dc, T} <- lists:zip(Dcs, lists:sublist(Words, length(Dcs))),
                               T =/= ?U64_MAX]).

%% ---------------------------------------------------------------------------
%% The engine-owned partition: materializer_vnode's ops cache in HBM.  Like
%% ops_cache-<P> it holds keys of every CRDT type (one device op log per
%% type, created with the type's first op); a read of a key that holds ops of
%% another type raises corrupted_ops_cache, as materialize_intern does
%% (src/clocksi_materializer.erl:190-191).
%% Cached = true: the snapshot cache lives on the device too (every type: the
%% set_aw / register_mv snapshot states stay on the device), read/5 is the
%% whole read/6; Cached = false: the reference's own ETS
%% snapshot cache stays, and read_from/7 is materialize/4 over the resident ops.
new_partition(Type, NKeys, Cached) ->
    {ok, Ps} = application:get_env(antidote, gpu_dcs),   % DC slots per clock (<= 256)
    part_open(ctx(), type_id(Type), Ps, NKeys, Cached).

%% update/2 -> op_insert_gc/3 (:621-647) on a cached partition, in the
%% reference's order: when the trigger of :635 holds, the GC read at the op's
%% snapshot time (:640) runs first, then the op is inserted.  Its OpSSCommit is
%% the snapshot_time with the commit DC set to the commit time
%% (src/clocksi_materializer.erl:224).  Returns {ok, OpId, GcRan}.  (With the
%% reference's ETS snapshot cache, the vnode checks part_gc_due/3 itself, runs
%% its own internal_read(..., true) -- whose snapshot_insert_gc calls gc/3 --
%% and then part_update/6.)
update(Part, Key, #clocksi_payload{type = Type, snapshot_time = SS, commit_time = {Dc, Ct},
                                   txid = TxId, op_param = Effect}) ->
    TypeId = type_id(Type),
    GcRan = case part_gc_due(Part, Key, TypeId) of
                true ->
                    case part_read(Part, Key, TypeId, dict:to_list(SS), ignore, true) of
                        {error, not_cached} ->
                            %% an uncached partition's GC read is the vnode's own
                            %% (its ETS snapshot cache): use part_update/6 there
                            erlang:error({update_needs_cached_partition, Key});
                        {error, no_snapshot} ->
                            %% no cached snapshot <= the op's snapshot time: the GC
                            %% read goes to the log, and its result is stored with
                            %% the GC on the device cache (internal_read(..., true),
                            %% :640 -> get_from_snapshot_log :416-419 ->
                            %% materialize_snapshot :466-509)
                            _ = read_from_log(Part, Key, Type, SS, ignore, true),
                            true;
                        _ -> true
                    end;
                false -> false
            end,
    case part_update(Part, Key, TypeId, dict:to_list(dict:store(Dc, Ct, SS)), TxId, Effect) of
        {ok, OpId, _} -> {ok, OpId, GcRan};
        Error -> Error
    end.

%% read/6 on a cached partition without the log fallback: {ok, Value} |
%% {error, no_snapshot} (the caller reads the log: get_from_snapshot_log,
%% :416-419; read/5 below does it) | {error, Reason}.
read_cached(Part, Key, Type, MinSnapshotTime, TxId) ->
    case part_read(Part, Key, type_id(Type), dict:to_list(MinSnapshotTime), TxId, false) of
        {ok, Value, _NewLastOp, _LastOpCt, _IsNewSS, _Count} -> {ok, Value};
        Other -> Other
    end.

%% read/6 with the log fallback (internal_read/7, :371-376, ShouldGc = false).
read(Part, Key, Type, MinSnapshotTime, TxId) ->
    case read_cached(Part, Key, Type, MinSnapshotTime, TxId) of
        {error, no_snapshot} -> read_from_log(Part, Key, Type, MinSnapshotTime, TxId, false);
        Other -> Other
    end.

%% get_from_snapshot_log (:416-419) + materialize_snapshot (:466-509) for a
%% cached partition: the key's ops from the partition's log
%% (logging_vnode:get_up_to_time), materialize/4 over them on the device
%% (per-call path), and -- for a GC read -- the result stored with its GC on
%% the device cache (part_store/8).  A log response is never the newest
%% snapshot (src/logging_vnode.erl:538-540), so a plain read stores nothing.
%% The reference's store cannot fail; a device store that does (the arena
%% re-pack out of memory, a clock wider than the partition) leaves the
%% snapshot uncached, which only costs a later read the log again.
read_from_log(Part, Key, Type, SnapshotTime, TxId, ShouldGc) ->
    LogId = log_utilities:get_logid_from_key(Key),
    Partition = log_utilities:get_key_partition(Key),
    case logging_vnode:get_up_to_time(Partition, LogId, SnapshotTime, Type, Key) of
        {error, Reason} -> {error, Reason};
        #snapshot_get_response{number_of_ops = 0, materialized_snapshot = Snapshot} ->
            {ok, Snapshot#materialized_snapshot.value};
        Resp ->
            case materialize(Type, TxId, SnapshotTime, Resp) of
                {error, Reason} -> {error, Reason};
                {ok, Value, _NewLastOp, ignore, _WasUpdated, _Count} -> {ok, Value};
                {ok, Value, NewLastOp, CommitTime, _WasUpdated, Count} ->
                    case ShouldGc of
                        true ->
                            case part_store(Part, Key, type_id(Type), dict:to_list(CommitTime),
                                            NewLastOp, Count, Value, true) of
                                ok -> ok;
                                {error, Why} ->
                                    logger:warning("gpu partition: snapshot of ~p not cached: ~p",
                                                   [Key, Why])
                            end;
                        false -> ok
                    end,
                    {ok, Value}
            end
    end.

%% materialize/4 over the partition's resident ops from a base snapshot the
%% caller's ETS snapshot cache selected: same result as
%% clocksi_materializer:materialize/4 ({ok, V, NewLastOp, LastOpCt, IsNewSS, Count}).
read_from(Part, Key, Type, MinSnapshotTime, SCT, TxId, BaseValue) ->
    Sct = case SCT of ignore -> ignore; _ -> dict:to_list(SCT) end,
    case part_materialize(Part, Key, type_id(Type), dict:to_list(MinSnapshotTime), Sct, TxId,
                          BaseValue) of
        {ok, V, H, Ct, NewSS, C} ->
            {ok, V, H, case Ct of ignore -> ignore; _ -> dict:from_list(Ct) end, NewSS, C};
        Other -> Other
    end.

%% snapshot_insert_gc's prune_ops + resize for one key (threshold = the
%% vectorclock:min of the kept snapshots, :523-527).
gc(Part, Key, Threshold) ->
    part_gc(Part, Key, dict:to_list(Threshold)).
