import sys; import os; R=os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0,R+'/tests'); sys.path.insert(0,R+'/dect-nr-plus-sdr_amd')
import numpy as np, test_gpu_parity as T, oracle_py as O, phy_fixtures as F, dnrp, torch
for name,snr in [("C2",10.0),("C3",30.0),("C4",30.0)]:
    for g_pcc,g_pdc,r1,r2,r in T._rx_case(name,snr):
        d=np.abs(g_pdc.astype(int)-r['pdc_llr'].astype(int)); dp=np.abs(g_pcc.astype(int)-r['pcc_llr'].astype(int))
        print(name,'pdc max',d.max(),'frac1 %.2e'%(d>0).mean(),'pcc max',dp.max(),'snr',r1.snr_dB,r['snr_pcc'],r2.snr_dB,r['snr_pdc'],'sto',r1.sto_fractional,r['sto'],'cfo',r1.cfo_fractional_rad, 'llr absmean', np.abs(g_pdc).mean())
rng=np.random.default_rng(0)
for name in ["C2","C3","C4"]:
    phy,ps,ops,ocf=T._ctx(name); sz=phy.packet_sizes(ps); S=sz['N_samples_packet_os_rs']
    _,_,pcc,pdc=T._tx_inputs(rng,2,sz)
    descs=[dnrp.TxDesc(0,100,1,5,1.0,0.3,0.01,0),dnrp.TxDesc(0,101,2,5,1.0,0.0,0.0,0)]
    iq=T._gpu_tx(phy,ps,descs,pcc,pdc,S)
    for i,d in enumerate(descs):
        ref,_=O.tx(ocf,ops,pcc[i],pdc[i],S,network_id=d.network_id,plcf_type=d.plcf_type,phase=float(np.float32(d.iq_phase_rad)),phase_inc=float(np.float32(d.iq_phase_increment_s2s_post_resampling_rad)))
        k=sz['N_samples_packet_no_GI_os_rs']
        print(name,i,[float(np.linalg.norm(iq[i,a,:k]-ref[a,:k])/np.linalg.norm(ref[a,:k])) for a in range(sz['N_TX'])])
